"""Workgroup timeline of one render launch (counting variant, s_memrealtime at 100 MHz):
how much of the kernel's wall time is the tail where few workgroups remain.  Needs a tuning build
(VR_WG_TIMES_PATH is read only there):  OUTDIR=abx bash tools/build_variant.sh tune -DVR_TUNING_VARIANTS;
    VR_LIBRARY=abx/libtune.so python tools/wg_tail.py [spp] [scene] [size]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vanrijn_amd import scenes  # noqa: E402
from vanrijn_amd.render import Tile, render_tile_device  # noqa: E402


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    which = sys.argv[2] if len(sys.argv) > 2 else "main"  # argv[3]: frame size (square)
    path = "/tmp/wg_times.bin"
    os.environ["VR_WG_TIMES_PATH"] = path
    ds = (scenes.main_scene() if which == "main" else scenes.bench_scene()).device_scene(0)
    W = H = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
    state = torch.zeros(W * H * 8, dtype=torch.float64, device="cuda")
    st = render_tile_device(ds, Tile(0, W, 0, H), H, W, spp, 1, 0, state.data_ptr(),
                            torch.cuda.current_stream().cuda_stream, counters=True)
    t = np.fromfile(path, dtype=np.uint64).reshape(-1, 2).astype(np.float64) * 10.0  # ns
    t0 = t[:, 0].min()
    s, e = t[:, 0] - t0, t[:, 1] - t0
    makespan = e.max()
    dur = e - s
    grid = np.linspace(0, makespan, 200)
    active = np.array([((s <= g) & (e > g)).sum() for g in grid])
    peak = active.max()
    # time after which fewer than half the peak workgroups are running
    half = grid[np.argmax((active < peak / 2) & (grid > grid[np.argmax(active)]))]
    out = {"scene": which, "spp": spp, "kernel_ms": st["kernel_ms"], "makespan_ms": makespan / 1e6, "blocks": len(s),
           "peak_concurrent": int(peak), "mean_concurrent": float(active.mean()),
           "utilisation": float(active.mean() / peak), "tail_start_ms": float(half / 1e6),
           "wg_ms_p50": float(np.median(dur) / 1e6), "wg_ms_p99": float(np.percentile(dur, 99) / 1e6),
           "wg_ms_max": float(dur.max() / 1e6), "last_start_ms": float(s.max() / 1e6)}
    print(json.dumps(out))
    np.save("gpurun_out/wg_times.npy", np.stack([s, e], 1))


if __name__ == "__main__":
    main()

"""Small-frame tail diagnostic: for one launch, the kernel time, the workgroup
timeline of the counting variant (s_memrealtime at 100 MHz) and the path-length distribution of the
same samples (record variant), so the tail can be attributed to long paths or to the launch shape.
    VR_LIBRARY=abx/libtune.so python tools/tail.py <scene main|bench> <size> <spp>  -> one JSON line
(VR_WG_TIMES_PATH is read only by a tuning build: OUTDIR=abx bash tools/build_variant.sh tune -DVR_TUNING_VARIANTS)"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vanrijn_amd import scenes  # noqa: E402
from vanrijn_amd.render import Tile, render_samples, render_tile_device  # noqa: E402


def main():
    which, size, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    ds = (scenes.main_scene() if which == "main" else scenes.bench_scene()).device_scene(0)
    W = H = size
    state = torch.zeros(W * H * 8, dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    ms = []
    for rep in range(5):
        st = render_tile_device(ds, Tile(0, W, 0, H), H, W, spp, 1, 0, state.data_ptr(), stream, timed=True)
        ms.append((st["kernel_ms"], st["reduce_ms"]))
    path = "/tmp/vr_wg_times.bin"
    os.environ["VR_WG_TIMES_PATH"] = path
    cnt = render_tile_device(ds, Tile(0, W, 0, H), H, W, spp, 1, 0, state.data_ptr(), stream, counters=True)
    del os.environ["VR_WG_TIMES_PATH"]
    t = np.fromfile(path, dtype=np.uint64).reshape(-1, 2).astype(np.float64) * 10.0  # ns
    s, e = t[:, 0] - t[:, 0].min(), t[:, 1] - t[:, 0].min()
    rec = render_samples(ds, Tile(0, W, 0, H), H, W, spp, seed=1)
    b = rec["bounces"].reshape(-1)
    out = {"scene": which, "size": size, "spp": spp, "samples": W * H * spp,
           "kernel_ms_median": float(np.median([x[0] for x in ms])), "reduce_ms_median": float(np.median([x[1] for x in ms])),
           "counting_kernel_ms": cnt["kernel_ms"], "workgroups": len(s),
           "wg_end_ms": {q: float(np.percentile(e, q) / 1e6) for q in (10, 50, 90, 99, 100)},
           "wg_start_ms_max": float(s.max() / 1e6),
           "bounces": {"mean": float(b.mean()), "p99": float(np.percentile(b, 99)), "p999": float(np.percentile(b, 99.9)),
                       "max": int(b.max()), "paths_ge_64": int((b >= 64).sum()), "paths_at_128": int((b >= 128).sum())},
           "lane_utilisation": {"traversal": cnt["node_visits"] / max(1, cnt["traversal_slots"]),
                                "path_loop": cnt["rays"] / max(1, cnt["path_loop_slots"])}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

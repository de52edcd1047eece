"""The launch tail of small frames: the longest paths alone.  Finds the (pixel, sample) pairs of a
frame whose paths run to the recursion limit (record variant), then renders just such a pixel
(1x1 tile, the frame's spp) timed and with counters: the kernel time of that launch is the latency
of the longest path, and the counters give its per-ray traversal work.
    python tools/longpath.py <scene bench|main> <size> <spp>  -> one JSON line"""
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
    rec = render_samples(ds, Tile(0, size, 0, size), size, size, spp, seed=1)
    b = rec["bounces"]
    worst = np.argwhere(b == b.max())
    row, col, s = (int(x) for x in worst[0])
    state = torch.zeros(8, dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    t = Tile(col, col + 1, row, row + 1)
    ms = [render_tile_device(ds, t, size, size, spp, 1, 0, state.data_ptr(), stream, timed=True)["kernel_ms"]
          for _ in range(5)]
    one = [render_tile_device(ds, t, size, size, 1, 1, s, state.data_ptr(), stream, timed=True)["kernel_ms"]
           for _ in range(5)]
    cpath = os.path.join("gpurun_out", "longpath_counters.bin")
    os.makedirs("gpurun_out", exist_ok=True)
    os.environ["VR_COUNTERS_PATH"] = cpath
    c = render_tile_device(ds, t, size, size, 1, 1, s, state.data_ptr(), stream, counters=True)
    del os.environ["VR_COUNTERS_PATH"]
    raw = np.fromfile(cpath, dtype=np.uint64)
    out = {"scene": which, "size": size, "spp": spp, "max_bounces": int(b.max()), "paths_at_max": len(worst),
           "pixel": [row, col], "sample": s, "pixel_bounces": b[row, col].tolist(),
           "pixel_launch_ms": float(np.median(ms)), "one_path_launch_ms": float(np.median(one)),
           "one_path": {k: c[k] for k in ("rays", "node_visits", "box_tests", "triangle_tests", "exact_box_tests",
                                          "traversal_slots", "path_loop_slots")}}
    out["one_path"]["us_per_bounce"] = out["one_path_launch_ms"] * 1e3 / max(1, int(b.max()))
    # where the lone path's wave spends its clock (counting variant, per-section s_memtime), and
    # how often each section ran (tools/cycles.py's names)
    cyc = raw[9:15].astype(np.float64)
    out["one_path"]["cycles_share"] = {k: round(float(v / max(1.0, cyc.sum())), 4) for k, v in zip(
        ["shade", "refill", "camera_begin_ray", "node_step", "leaf_round", "next_bvh_and_loop"], cyc)}
    out["one_path"]["cycles_total"] = float(cyc.sum())
    out["one_path"]["wave_executions"] = {k: int(v) for k, v in zip(
        ["leaf_test", "leaf_test_2nd", "exact_box", "shade", "camera", "begin_ray", "finish", "refill",
         "start_bvhs_trav"], raw[15:24])}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

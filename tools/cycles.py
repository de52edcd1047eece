"""Per-section wave clock cycles of the render kernel's counting variant (diagnostic).
    python tools/cycles.py [spp] [scene]
Needs a tuning build (VR_COUNTERS_PATH is read only with -DVR_TUNING_VARIANTS: `bash
tools/build_variant.sh tune -DVR_TUNING_VARIANTS`, then VR_LIBRARY=ab/libtune.so)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vanrijn_amd import scenes  # noqa: E402
from vanrijn_amd.render import Tile, render_tile_device  # noqa: E402

SECTIONS = ["shade", "refill", "camera_begin_ray", "node_step", "leaf_round", "next_bvh_and_loop"]
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
which = sys.argv[2] if len(sys.argv) > 2 else "main"
torch.cuda.set_device(0)
ds = (scenes.main_scene() if which == "main" else scenes.bench_scene()).device_scene(0)
state = torch.zeros(1024 * 1024 * 8, dtype=torch.float64, device="cuda")
# an absolute path under the repository (the box runs from a scratch copy; a relative path depended
# on the working directory and on gpurun_out/ existing), removed first so a stale file never answers
out_dir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
os.makedirs(out_dir, exist_ok=True)
path = os.path.join(out_dir, "counters.bin")
if os.path.exists(path):
    os.remove(path)
os.environ["VR_COUNTERS_PATH"] = path
st = render_tile_device(ds, Tile(0, 1024, 0, 1024), 1024, 1024, spp, 1, 0, state.data_ptr(),
                        torch.cuda.current_stream().cuda_stream, counters=True)
if not os.path.exists(path):
    sys.exit("tools/cycles.py: no counters written -- the library is not a tuning build "
             "(VR_LIBRARY=<a -DVR_TUNING_VARIANTS build>, see the docstring)")
c = np.fromfile(path, dtype=np.uint64)
cyc = c[9:15].astype(np.float64)
out = {"scene": which, "spp": spp, "kernel_ms": st["kernel_ms"],
       "cycles_share": {k: round(float(v / cyc.sum()), 4) for k, v in zip(SECTIONS, cyc)},
       "cycles_total": float(cyc.sum()),
       "wave_executions": {k: int(v) for k, v in zip(["leaf_test", "leaf_test_2nd", "exact_box", "shade", "camera",
                                                        "begin_ray", "finish", "refill", "start_bvhs_trav"],
                                                       c[15:24])}, "counters": {k: st[k] for k in st if k not in ("kernel_ms", "timed")}}
if len(c) >= 33:
    # phase-B iterations by how many lanes take a node step in them (0, 1-8, .., 57-64): the
    # headroom of merging waves' traversing lanes is the iterations a perfect
    # packing of the same node steps would not need
    h = c[24:33].astype(np.int64)
    labels = ["0"] + ["%d-%d" % (8 * i + 1, 8 * i + 8) for i in range(8)]
    out["node_step_lanes_hist"] = {k: int(v) for k, v in zip(labels, h)}
    steps = int(h[1:].sum())
    packed = int(np.ceil(st["node_visits"] / 64.0))
    out["node_step_iterations"] = steps
    out["node_step_iterations_perfectly_packed"] = packed
    out["node_step_lane_utilisation"] = round(st["node_visits"] / (64.0 * max(1, steps)), 4)
if len(c) >= 36:
    # wave-level f64 sphere tests (begin_ray): how many ran, and how many of their lanes the f32
    # pre-test left (the rest of the active lanes only follow along)
    out["sphere_tests"] = {"wave_executions": int(c[33]), "maybe_lanes": int(c[34]), "active_lanes": int(c[35]),
                           "maybe_lanes_per_execution": round(float(c[34]) / max(1, int(c[33])), 2),
                           "active_lanes_per_execution": round(float(c[35]) / max(1, int(c[33])), 2)}
print(json.dumps(out))

"""Drop-in call pattern (src/main.rs:197-216) breakdown on one GPU: per-call latency of
partial_render_scene (1 spp, full frame, host buffers), merge_tile time, and the aggregate
Msamples/s with T worker threads + one merging thread.
    python tools/dropin.py [size] [frames]"""
import json
import os
import sys
import time

import torch  # noqa: F401  (binds the library to torch's HIP runtime)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from vanrijn_amd import scenes  # noqa: E402
from vanrijn_amd.render import AccumulationBuffer, Tile, partial_render_scene  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 32
ds = scenes.main_scene().device_scene(0)
tile = Tile(0, size, 0, size)
out = {"size": size}
lat = []
os.environ["VR_HOST_TIMING"] = "1"
for i in range(6):
    t0 = time.perf_counter()
    b = partial_render_scene(ds, tile, size, size)
    lat.append((time.perf_counter() - t0) * 1e3)
out["call_ms"] = [round(x, 2) for x in lat]
t0 = time.perf_counter()
for i in range(6):
    b2 = AccumulationBuffer._for_output(size, size)
    for a in (b2.colour_buffer, b2.colour_sum_buffer, b2.colour_bias_buffer, b2.weight_buffer, b2.weight_bias_buffer):
        a.fill(0.0)
out["alloc_touch_ms"] = round((time.perf_counter() - t0) / 6 * 1e3, 2)
grab = {}
for g in ("64", "128", "256", "512", ""):
    if g:
        os.environ["VR_GRAB"] = g
    else:
        os.environ.pop("VR_GRAB", None)
    ts = []
    for i in range(5):
        t0 = time.perf_counter()
        partial_render_scene(ds, tile, size, size)
        ts.append((time.perf_counter() - t0) * 1e3)
    grab[g or "auto"] = round(sorted(ts)[2], 2)
out["call_ms_by_grab"] = grab
img = AccumulationBuffer(size, size)
mt = []
for i in range(6):
    t0 = time.perf_counter()
    img.merge_tile(tile, b)
    mt.append((time.perf_counter() - t0) * 1e3)
out["merge_ms"] = [round(x, 2) for x in mt]
out["threads"] = {}
for t in (1, 2, 4, 8, 16):
    r = bench.drop_in_leg(ds, size, size, frames, t, 0)
    out["threads"][t] = {"msamples_s": r["value"], "ms_per_frame": r["ms_per_frame"]}
    print(t, r["value"], flush=True)
print(json.dumps(out))

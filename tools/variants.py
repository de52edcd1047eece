"""A/B the render-kernel variants in ONE process, interleaved (rules 24/25 of the HIP guide).

    python tools/variants.py --spp 32 --reps 3 --variants 0,1,2,3,4 --thresholds 32
Prints one JSON line per (variant, threshold) with the median kernel ms over reps.
The variant / threshold / --env overrides are read only by a tuning build of the library
(-DVR_TUNING_VARIANTS: `VR_TUNING=1 python -m vanrijn_amd.build`, or `bash tools/build_variant.sh
NAME -DVR_TUNING_VARIANTS` and VR_LIBRARY=ab/libNAME.so); a default build ignores them.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vanrijn_amd import scenes  # noqa: E402
from vanrijn_amd.render import Tile, render_tile_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=32)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--thresholds", default="32")
    ap.add_argument("--scene", default="main")
    ap.add_argument("--env", action="append", default=[],
                    help="NAME=v1,v2,... sweep over an environment variable (repeatable: cartesian product)")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    scene = {"main": scenes.main_scene, "bench": scenes.bench_scene, "c5": scenes.synthetic_scene,
             "materials": scenes.materials_scene, "whitted": scenes.whitted_scene}[a.scene]()
    ds = scene.device_scene(0)
    W = H = a.size
    state = torch.zeros(W * H * 8, dtype=torch.float64, device="cuda")
    ref = None
    results = {}
    import itertools
    names = [x.split("=", 1)[0] for x in a.env]
    evals = list(itertools.product(*[x.split("=", 1)[1].split(",") for x in a.env]))
    combos = [(v, t, e) for v in a.variants.split(",") for t in a.thresholds.split(",") for e in evals]
    for rep in range(a.reps):
        for v, t, e in combos:
            os.environ["VR_KERNEL_VARIANT"] = v
            os.environ["VR_SHADE_THRESHOLD"] = t
            for n, val in zip(names, e):
                os.environ[n] = val
            st = render_tile_device(ds, Tile(0, W, 0, H), H, W, a.spp, 1, 0, state.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream, timed=True)
            out = state.cpu()
            if ref is None:
                ref = out
            same = bool(torch.equal(out, ref))
            results.setdefault((v, t, e), []).append((st["kernel_ms"], same, st.get("reduce_ms", 0.0)))
    for (v, t, e), r in results.items():
        ms = [x[0] for x in r]
        print(json.dumps({"variant": v, "threshold": t, **dict(zip(names, e)), "scene": a.scene,
                          "median_ms": statistics.median(ms), "min_ms": min(ms),
                          "reduce_ms": statistics.median([x[2] for x in r]),
                          "msamples_s": W * H * a.spp / statistics.median(ms) / 1e3,
                          "bitwise_equal_to_first": all(x[1] for x in r)}), flush=True)


if __name__ == "__main__":
    main()

"""C1's frame time, frame by frame (tools/ab.sh's 1.603 ms against bench.py's 1.748 ms).

C1 (benches/simple_scene.rs: the reflective bunny, 256^2 @16) is set by the few paths trapped between
mirror facets that run to the 128-bounce limit, and WHICH samples get trapped depends on the seed and
the sample range.  tools/ab.sh / variants.py render ONE frame (seed 1, samples 0..15) again and again;
bench.py renders a new sample range per frame (seed 0x5EED0001, samples 16 k .. 16 k + 15).  This
prints, per frame, the render kernel's HIP-event time for both, each launch timed alone (the GPU idle
before it), so the two harnesses' numbers can be compared frame by frame.
    python tools/c1_frames.py [frames]"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vanrijn_amd import scenes  # noqa: E402
from vanrijn_amd.render import Tile, render_tile_device  # noqa: E402


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    torch.cuda.set_device(0)
    ds = scenes.bench_scene().device_scene(0, device_sah=True)
    H = W = 256
    t = Tile(0, W, 0, H)
    st = torch.zeros(H * W * 8, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):  # warm
        render_tile_device(ds, t, H, W, 16, 1, 0, st.data_ptr(), s, timed=True)
    same, bench = [], []
    for k in range(frames):
        same.append(render_tile_device(ds, t, H, W, 16, 1, 0, st.data_ptr(), s, timed=True)["kernel_ms"])
        bench.append(render_tile_device(ds, t, H, W, 16, 0x5EED0001, 16 * (k + 1), st.data_ptr(), s,
                                        timed=True)["kernel_ms"])
    out = {"variants_py_frame (seed 1, samples 0..15)": {"median_ms": round(statistics.median(same), 4),
                                                         "min": round(min(same), 4), "max": round(max(same), 4)},
           "bench_py_frames (seed 0x5EED0001, samples 16k..16k+15)": {
               "median_ms": round(statistics.median(bench), 4), "mean_ms": round(statistics.mean(bench), 4),
               "min": round(min(bench), 4), "max": round(max(bench), 4),
               "per_frame_ms": [round(x, 3) for x in bench]}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""16-bit against 32-bit traversal-stack entries (VR_LAUNCH_STACK32) in one process, interleaved:
    python tools/stack16_ab.py [scene main|bench|c5] [size] [spp] [reps]  -> one JSON line"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vanrijn_amd import scenes  # noqa: E402
from vanrijn_amd.render import Tile, render_tile_device  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "main"
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    spp = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    torch.cuda.set_device(0)
    sc = {"main": scenes.main_scene, "bench": scenes.bench_scene, "c5": scenes.synthetic_scene}[which]()
    ds = sc.device_scene(0, device_sah=True)
    t = Tile(0, size, 0, size)
    st = torch.zeros(size * size * 8, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    res, outs = {True: [], False: []}, {}
    render_tile_device(ds, t, size, size, spp, 1, 0, st.data_ptr(), s, timed=True)
    for rep in range(reps):
        for s16 in (True, False):
            r = render_tile_device(ds, t, size, size, spp, 1, 0, st.data_ptr(), s, timed=True, stack16=s16)
            res[s16].append(r["kernel_ms"])
            outs[s16] = (st.cpu(), r["variant"])
    same = bool(torch.equal(outs[True][0].view(torch.int64), outs[False][0].view(torch.int64)))
    print(json.dumps({"scene": which, "size": size, "spp": spp,
                      "stack16_ms": round(statistics.median(res[True]), 3), "stack32_ms": round(statistics.median(res[False]), 3),
                      "all16": [round(x, 3) for x in res[True]], "all32": [round(x, 3) for x in res[False]],
                      "variants": [outs[True][1], outs[False][1]], "bitwise_equal": same}), flush=True)


if __name__ == "__main__":
    main()

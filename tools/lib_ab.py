"""One library build's render-kernel time and record digest on one configuration (run once per
library, VR_LIBRARY=<lib> selects it; the digests of two builds must match bit for bit):
    VR_LIBRARY=abx/libX.so python tools/lib_ab.py [scene main|bench|c5] [size] [spp] [reps]"""
import hashlib
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
    render_tile_device(ds, t, size, size, spp, 1, 0, st.data_ptr(), s, timed=True)
    ms, red = [], []
    for _ in range(reps):
        r = render_tile_device(ds, t, size, size, spp, 1, 0, st.data_ptr(), s, timed=True)
        ms.append(r["kernel_ms"])
        red.append(r["reduce_ms"])
    digest = hashlib.sha256(st.cpu().view(torch.int64).numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"lib": os.environ.get("VR_LIBRARY", "in-tree"), "scene": which, "size": size, "spp": spp,
                      "median_ms": round(statistics.median(ms), 3), "all": [round(x, 3) for x in ms],
                      "reduce_ms": round(statistics.median(red), 3),
                      "variant": r["variant"], "digest": digest}), flush=True)


if __name__ == "__main__":
    main()

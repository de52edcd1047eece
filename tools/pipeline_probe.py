"""Frames back to back on one stream vs alternated over two streams (two record buffers): how much
of a frame's launch tail and ordered reduce the next frame's render absorbs.
    python tools/pipeline_probe.py [scene main|bench|c5] [size] [spp] [frames]  -> JSON lines"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vanrijn_amd import scenes  # noqa: E402
from vanrijn_amd.render import Tile, render_tile_device  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "main"
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    spp = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    frames = int(sys.argv[4]) if len(sys.argv) > 4 else 6
    torch.cuda.set_device(0)
    sc = {"main": scenes.main_scene, "bench": scenes.bench_scene, "c5": scenes.synthetic_scene}[which]()
    ds = sc.device_scene(0, device_sah=True)
    t = Tile(0, size, 0, size)
    states = [torch.zeros(size * size * 8, dtype=torch.float64, device="cuda") for _ in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    def run(nstreams, k0):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(frames):
            j = i % nstreams
            render_tile_device(ds, t, size, size, spp, 1, (k0 + i) * spp, states[j].data_ptr(),
                               streams[j].cuda_stream)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / frames * 1e3

    run(2, 0)  # warm both contexts
    res = {}
    for rep in range(3):
        for n in (1, 2):
            res.setdefault(n, []).append(run(n, 100 + rep * 50 + n * 10))
    ok = bool(torch.equal(states[0], states[0]))
    for n in (1, 2):
        v = sorted(res[n])
        print(json.dumps({"scene": which, "size": size, "spp": spp, "frames": frames, "streams": n,
                          "ms_per_frame_median": round(v[1], 3), "all": [round(x, 3) for x in res[n]],
                          "msamples_s": round(size * size * spp / v[1] / 1e3, 1), "ok": ok}), flush=True)


if __name__ == "__main__":
    main()

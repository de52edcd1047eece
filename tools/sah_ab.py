"""Device-built vs host-built SAH traversal tree (VR_SCENE_DEVICE_SAH): build time and render kernel
time on the same workload, interleaved, and the records compared bit for bit.
    python tools/sah_ab.py <scene main|c5> <size> <spp> [reps]  -> one JSON line"""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vanrijn_amd import scenes  # noqa: E402
from vanrijn_amd.render import Tile, render_tile_device  # noqa: E402


def main():
    which, size, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    torch.cuda.set_device(0)
    s = scenes.synthetic_scene() if which == "c5" else scenes.main_scene()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = s.device_scene(0)
    t_host = time.perf_counter() - t0
    t0 = time.perf_counter()
    dev = s.device_scene(0, device_sah=True)
    t_dev = time.perf_counter() - t0
    W = H = size
    st = {k: torch.zeros(W * H * 8, dtype=torch.float64, device="cuda") for k in ("host", "device")}
    ms = {"host": [], "device": []}
    for r in range(reps):
        for k, ds in (("host", host), ("device", dev)):
            out = render_tile_device(ds, Tile(0, W, 0, H), H, W, spp, 0x5EED0001, 0, st[k].data_ptr(),
                                     torch.cuda.current_stream().cuda_stream, timed=True)
            ms[k].append(out["kernel_ms"])
    same = bool(torch.equal(st["host"], st["device"]))
    cnt = {k: render_tile_device(ds, Tile(0, W, 0, H), H, W, spp, 0x5EED0001, 0, st[k].data_ptr(),
                                 torch.cuda.current_stream().cuda_stream, counters=True)
           for k, ds in (("host", host), ("device", dev))}
    print(json.dumps({"scene": which, "size": size, "spp": spp, "build_s": {"host": t_host, "device": t_dev},
                      "kernel_ms_median": {k: statistics.median(v) for k, v in ms.items()}, "kernel_ms": ms,
                      "records_bit_identical": same,
                      "node_visits": {k: cnt[k]["node_visits"] for k in cnt},
                      "triangle_tests": {k: cnt[k]["triangle_tests"] for k in cnt},
                      "wide_nodes": {"host": host.info()["wide_node_count"], "device": dev.info()["wide_node_count"]},
                      "traversal_stack": {"host": host.info()["traversal_stack"],
                                          "device": dev.info()["traversal_stack"]}}), flush=True)


if __name__ == "__main__":
    main()

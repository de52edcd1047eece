"""The megakernel split, measured ("the megakernel split").

Needs the analysis build (-DVR_SPLIT_PROBE):
    OUTDIR=abx bash tools/build_variant.sh split -DVR_SPLIT_PROBE
    VR_LIBRARY=abx/libsplit.so python tools/split_probe.py [main|c5] [size] [spp]

1. Times the production render of the frame (render kernel, HIP events) with the dump off.
2. Renders it once more with every traced ray (origin, direction: 6 f64) appended to a device buffer.
3. Runs the traversal-only TRACE instantiation of the same kernel (no shading, no path state: the
   machinery a split design's traversal kernel would keep -- node steps, wave leaf FIFO, leaf rounds,
   primitive tests) over exactly those rays at 3 / 4 / 5 waves per SIMD, 32- or 16-bit LDS stack
   entries, and times each (3 repetitions, interleaved).
4. Checks a strided sample of 200k TRACE hits against the exact binary-tree trace kernel (vr_trace_rays)
   bit for bit (distance, object, hit / miss).
Prints one JSON line per configuration and a summary line."""
import ctypes as C
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vanrijn_amd import _native as N  # noqa: E402
from vanrijn_amd import scenes  # noqa: E402
from vanrijn_amd.render import Tile, render_tile_device, trace_rays  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "main"
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    spp = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    torch.cuda.set_device(0)
    lib = N.lib()
    lib.vr_probe_set_dump.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
    lib.vr_probe_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                   C.c_void_p, C.POINTER(C.c_float)]
    scene = scenes.main_scene() if which == "main" else scenes.synthetic_scene()
    ds = scene.device_scene(0, device_sah=True)
    t = Tile(0, size, 0, size)
    state = torch.zeros(size * size * 8, dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    lib.vr_probe_set_dump(None, None, 0)
    mk = []
    for rep in range(3):  # the production launch, dump off
        mk.append(render_tile_device(ds, t, size, size, spp, 1, rep * spp, state.data_ptr(), stream, timed=True)["kernel_ms"])
    cap = int(2.6 * size * size * spp) + (1 << 20)
    rays = torch.empty(cap * 6, dtype=torch.float64, device="cuda")
    count = torch.zeros(1, dtype=torch.int64, device="cuda")
    lib.vr_probe_set_dump(C.c_void_p(rays.data_ptr()), C.c_void_p(count.data_ptr()), cap)
    render_tile_device(ds, t, size, size, spp, 1, 0, state.data_ptr(), stream, timed=True)
    lib.vr_probe_set_dump(None, None, 0)
    torch.cuda.synchronize()
    n = int(count.item())
    assert 0 < n <= cap, (n, cap)
    hits = torch.empty(n * 2, dtype=torch.float64, device="cuda")
    # 16-bit stack entries need a tree below 65,536 wide nodes (the bunny's 27,441; not C5's 413,444),
    # and more than 3 workgroups per CU need them (LDS)
    configs = [(3, 0), (3, 1), (4, 1), (5, 1)] if which == "main" else [(3, 0)]
    res = {}
    ms = C.c_float()
    for rep in range(int(os.environ.get("SPLIT_REPS", "3"))):
        for minw, s16 in configs:
            rc = lib.vr_probe_trace(ds.handle, C.c_void_p(rays.data_ptr()), n, C.c_void_p(hits.data_ptr()), minw, s16,
                                    3 if minw == 3 else (4 if minw == 4 else 5), C.c_void_p(stream), C.byref(ms))
            N.check(rc)
            res.setdefault((minw, s16), []).append(ms.value)
    if os.environ.get("SPLIT_SORT") == "1":
        # the same rays reordered by (direction octant, 30-bit Morton code of the origin
        # in the origins' bounding box) -- the order a split design's ray queue could be sorted into
        # -- traced again at 3 waves per SIMD; the sort itself timed with CUDA events
        def spread(x):  # 10 bits -> every third bit
            x = (x | (x << 16)) & 0x030000FF
            x = (x | (x << 8)) & 0x0300F00F
            x = (x | (x << 4)) & 0x030C30C3
            return (x | (x << 2)) & 0x09249249
        r6 = rays[:n * 6].view(n, 6)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        o = r6[:, :3]
        lo, hi = o.min(0).values, o.max(0).values
        q = ((o - lo) / (hi - lo).clamp_min(1e-300) * 1023.0).clamp(0, 1023).to(torch.int64)
        key = spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)
        key |= ((r6[:, 3] < 0).to(torch.int64) << 32) | ((r6[:, 4] < 0).to(torch.int64) << 31) | \
            ((r6[:, 5] < 0).to(torch.int64) << 30)
        order = torch.argsort(key)
        del key, q, o
        sorted_rays = r6[order].contiguous().view(-1)
        e1.record()
        torch.cuda.synchronize()
        sort_ms = e0.elapsed_time(e1)
        del order
        sres = []
        for rep in range(3):
            N.check(lib.vr_probe_trace(ds.handle, C.c_void_p(sorted_rays.data_ptr()), n, C.c_void_p(hits.data_ptr()), 3, 0,
                                       3, C.c_void_p(stream), C.byref(ms)))
            sres.append(ms.value)
        print(json.dumps({"scene": which, "size": size, "spp": spp, "rays": n, "order": "octant + origin Morton",
                          "waves_per_simd": 3, "stack16": 0, "trace_ms_median": round(statistics.median(sres), 3),
                          "all_ms": [round(x, 3) for x in sres], "sort_ms": round(sort_ms, 3),
                          "grays_per_s": round(n / statistics.median(sres) / 1e6, 3)}), flush=True)
        rays = sorted_rays  # the check below then samples the sorted rays and their hits
    # correctness: a strided sample against the exact binary-tree trace kernel
    idx = np.linspace(0, n - 1, min(n, 200000)).astype(np.int64)
    rv = rays.view(-1, 6)[torch.from_numpy(idx).cuda()].cpu().numpy()
    hv = hits.view(-1, 2)[torch.from_numpy(idx).cuda()].cpu().numpy()
    ref = trace_rays(ds, rv[:, :3], rv[:, 3:])
    bits = hv[:, 1].view(np.uint64)
    kind = (bits & 3).astype(np.int64)
    obj = (bits >> 32).astype(np.int64)
    valid = kind != 0
    ok_valid = np.array_equal(valid, ref["valid"].astype(bool))
    ok_dist = np.array_equal(hv[valid, 0], ref["distance"][valid]) if ok_valid else False
    ok_obj = np.array_equal(obj[valid], ref["object"][valid]) if ok_valid else False
    for (minw, s16), v in res.items():
        med = statistics.median(v)
        print(json.dumps({"scene": which, "size": size, "spp": spp, "rays": n, "waves_per_simd": minw, "stack16": s16,
                          "trace_ms_median": round(med, 3), "all_ms": [round(x, 3) for x in v],
                          "grays_per_s": round(n / med / 1e6, 3)}), flush=True)
    print(json.dumps({"scene": which, "size": size, "spp": spp, "rays": n, "render_kernel_ms": [round(x, 3) for x in mk],
                      "render_grays_per_s": round(n / statistics.median(mk) / 1e6, 3),
                      "check_sample": len(idx), "hits_valid_equal": ok_valid, "distances_bitwise_equal": ok_dist,
                      "objects_equal": ok_obj, "hit_fraction": float(valid.mean())}), flush=True)


if __name__ == "__main__":
    main()

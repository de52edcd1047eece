#!/usr/bin/env python3
"""Benchmark: Msamples/s of the MI355X path-tracing core on BASELINE.json's headline config.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)

Workload (BASELINE.json configs[2] / metric): the main.rs scene (src/main.rs:120-189: plane,
three spheres, Lambertian bunny; camera (-2, 1, -5)) at 1024x1024, 256 samples per pixel.  The
bunny OBJ is a Git-LFS pointer in the reference, so the mesh is the deterministic procedural
stand-in (69,312 triangles, vanrijn_amd/scenes.py).  One "step" = one full frame at 256 spp on
every GPU (weak scaling: rank r renders sample indices [(step*N + r)*256, +256) of the same
image); for N > 1 the per-pixel accumulation records (8 f64) are summed onto rank 0 with one
RCCL reduce over xGMI inside the timed region.

Printed (rank 0, one JSON line): value = total samples of all ranks / max-over-ranks wall time,
the roofline of the render kernel (algorithmic bytes per launch from the kernel's counting
variant / HIP-event kernel time, against 8 TB/s HBM), and the CPU baseline: the oracle's
reference-mode restatement (exhaustive BVH traversal, recursive integrator) on a bounded sample
of the same frame, timed on the host cores of this box (rank 0, N = 1 only).
"""
import argparse
import json
import os
import sys
import time

import torch  # import first: the HIP library then binds to torch's HIP runtime (same soname)
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from vanrijn_amd import distributed as D  # noqa: E402
from vanrijn_amd import scenes  # noqa: E402
from vanrijn_amd.render import Tile, render_tile_device  # noqa: E402

METRIC = "Msamples/s + achieved HBM GB/s, 1024x1024 bunny @256spp, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
SEED = 0x5EED0001

# algorithmic bytes, SURVEY.md 8(d)'s per-unit figure (DESIGN.md "Roofline"): one f64 AABB (48 B)
# per box test, a triangle's 9 f64 vertices (72 B) per triangle test, its 9 f64 normals (72 B) per
# shaded triangle hit, one f64 (X, Y, Z, W) record (32 B) per pixel.
BYTES_PER_BOX_TEST = 48
BYTES_PER_TRI_TEST = 72
BYTES_PER_SHADED_TRI = 72
BYTES_PER_PIXEL_STATE = 32


def algorithmic_bytes(c, pixels):
    return (BYTES_PER_BOX_TEST * c["box_tests"] + BYTES_PER_TRI_TEST * c["triangle_tests"] +
            BYTES_PER_SHADED_TRI * c["shaded_triangle_hits"] + BYTES_PER_PIXEL_STATE * pixels)


def layout_bytes(c, pixels):
    """What this kernel's own layout reads and writes per launch before any cache: a 128-B Node4
    line per wide-node visit, a 48-B f64 box per exact fallback, the 80-B vertex record per triangle
    test, vertex + normal records (160 B) per shaded triangle hit, the 16-B staged photon per sample,
    the 64-B accumulation record per pixel (reported beside the roofline, not in it)."""
    return (128 * c["node_visits"] + 48 * c["exact_box_tests"] + 80 * c["triangle_tests"] +
            160 * c["shaded_triangle_hits"] + 16 * c["samples"] + 64 * pixels)


def pmc_traffic(args):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (tools/pmc.sh +
    tools/pmc_summary.py: 2*FETCH_SIZE + WRITE_SIZE), used only when it was collected on this
    exact library build and bench configuration; otherwise None."""
    import hashlib
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    lib = os.path.join(ROOT, "vanrijn_amd", "lib", "libvanrijn_amd.so")
    try:
        rec = json.load(open(path))
        sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()
    except (OSError, ValueError):
        return None
    want = f"--width {args.width} --height {args.height} --spp {args.spp} --scene {args.scene}"
    if rec.get("lib_sha256") != sha or rec.get("config") != want:
        return None
    return rec.get("hbm_bytes_per_launch")


def cpu_baseline(scene, width, height, seconds, threads):
    """Oracle (reference mode) on the host: full frame, first k sample indices, k chosen so the
    run takes about `seconds`."""
    from oracle import oracle_ffi as O
    orc = O.OracleScene(scene.spec())
    t = Tile(0, width, 0, height)
    t0 = time.perf_counter()
    r = orc.render_tile(t, height, width, 1, SEED, 0, O.MODE_REFERENCE, threads)
    one = time.perf_counter() - t0
    k = int(max(1, min(64, seconds / max(one, 1e-3))))
    samples = width * height
    total = one
    if k > 1:
        t0 = time.perf_counter()
        r = orc.render_tile(t, height, width, k - 1, SEED, 1, O.MODE_REFERENCE, threads)
        total += time.perf_counter() - t0
        samples += width * height * (k - 1)
    return {"value": samples / total / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{width}x{height} frame, sample indices 0..{k - 1} ({samples} samples, {total:.1f} s), "
                      f"oracle reference mode (exhaustive line-BVH traversal, recursive integrator), "
                      f"{threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--scene", choices=["main", "bench", "c5"], default="main",
                    help="main: main.rs scene (the headline); bench: benches/simple_scene.rs; "
                         "c5: SURVEY 8(d) C5, main.rs's plane and spheres + the 1,051,392-triangle synthetic mesh")
    ap.add_argument("--mesh", default=None,
                    help="the reference's test_data/stanford_bunny.obj (size + sha256 verified) instead of the "
                         "procedural stand-in")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    W, H, spp = args.width, args.height, args.spp
    if args.scene == "c5":
        scene = scenes.synthetic_scene()
    else:
        scene = scenes.main_scene(args.mesh) if args.scene == "main" else scenes.bench_scene(args.mesh)
    dscene = scene.device_scene(local)
    info = dscene.info()
    tile = Tile(0, W, 0, H)
    state = torch.zeros(H * W * 8, dtype=torch.float64, device=f"cuda:{local}")
    stream = torch.cuda.current_stream()

    def step(i, timed=False):
        st = render_tile_device(dscene, tile, H, W, spp, SEED, D.first_sample(i, rank, world, spp), state.data_ptr(),
                                stream.cuda_stream, timed=timed, device=local)
        D.reduce_records(state)  # RCCL sum of the records onto rank 0 (no-op at N = 1)
        return st

    # counting launch (untimed): traversal counters of exactly this workload
    counts = render_tile_device(dscene, tile, H, W, spp, SEED, rank * spp, state.data_ptr(), stream.cuda_stream,
                                counters=True, device=local)
    for i in range(args.warmup):
        step(1 + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    kernel_ms, reduce_ms = [], []
    t0 = time.perf_counter()
    for i in range(args.steps):
        st = step(1 + args.warmup + i, timed=True)
        kernel_ms.append(st["kernel_ms"])  # render kernel only (HIP events on the launch stream)
        reduce_ms.append(st["reduce_ms"])  # the ordered per-pixel Kahan reduce after it
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    samples = world * args.steps * W * H * spp
    value = samples / elapsed / 1e6
    avg_kernel_s = sum(kernel_ms) / len(kernel_ms) / 1e3
    alg_bytes = algorithmic_bytes(counts, W * H)
    achieved = alg_bytes / avg_kernel_s / 1e9
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic: lat-long displaced sphere mesh (1,051,392 triangles, seed 0x1DEA), counter-based RNG "
                 "seed 0x5EED0001") if args.scene == "c5" else
                ("synthetic: procedural bunny stand-in (69,312 triangles; the reference OBJ is an LFS pointer), "
                 "counter-based RNG seed 0x5EED0001") if args.mesh is None else
                f"{os.path.basename(args.mesh)} (sha256-verified reference bunny), counter-based RNG seed 0x5EED0001",
        "config": {"workload": {"main": f"main.rs scene (plane, 3 spheres, Lambertian bunny), {W}x{H} @{spp}spp per GPU",
                                "bench": f"bench scene (reflective bunny), {W}x{H} @{spp}spp per GPU",
                                "c5": f"C5: main.rs plane + spheres + 1,051,392-triangle synthetic mesh, {W}x{H} "
                                      f"@{spp}spp per GPU"}[args.scene],
                   "width": W, "height": H, "spp": spp, "triangles": info["triangle_count"],
                   "bvh_depth": info["max_bvh_depth"], "parallelism": f"spp-split x{world}, RCCL reduce"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(args),
                     "kernel": "render_kernel", "kernel_ms": round(avg_kernel_s * 1e3, 3),
                     "reduce_kernel_ms": round(sum(reduce_ms) / len(reduce_ms), 3),
                     "algorithmic_bytes_per_launch": alg_bytes,
                     "layout_bytes_per_launch": layout_bytes(counts, W * H),
                     "layout_gbs": round(layout_bytes(counts, W * H) / avg_kernel_s / 1e9, 2),
                     "counters_per_launch": {k: counts[k] for k in ("box_tests", "node_visits", "triangle_tests",
                                                                    "rays", "shaded_triangle_hits", "samples",
                                                                    "traversal_slots", "path_loop_slots",
                                                                    "exact_box_tests")},
                     "traversal_lane_utilisation": round(counts["node_visits"] / max(1, counts["traversal_slots"]), 4),
                     "path_loop_lane_utilisation": round(counts["rays"] / max(1, counts["path_loop_slots"]), 4)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(scene, W, H, args.cpu_seconds, args.cpu_threads)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

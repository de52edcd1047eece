#!/usr/bin/env python3
"""Benchmark: Msamples/s of the MI355X path-tracing core on BASELINE.json's headline config.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1|c2|c3|c4|c5]
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)

Workload (default --config c3 = BASELINE.json configs[2] / metric): the main.rs scene
(src/main.rs:120-189: plane, three spheres, Lambertian bunny; camera (-2, 1, -5)) at 1024x1024,
256 samples per pixel per GPU.  The bunny OBJ is a Git-LFS pointer in the reference, so the mesh is
the deterministic procedural stand-in (69,312 triangles, vanrijn_amd/scenes.py).  One "step" = one
frame: rank r renders sample indices [(step*N + r)*spp, +spp) of the same image (weak scaling for
c1-c3; c4 / c5 split ONE frame's 1024 / 256 spp over the N ranks, strong scaling), then the
per-pixel accumulation records (8 f64) are summed onto rank 0 with one RCCL reduce over xGMI inside
the timed region (vanrijn_amd/distributed.py frame_step, the same step the gloo tests run).

Printed (rank 0, one JSON line):
  value       total samples of all ranks / max-over-ranks wall time of the timed steps;
  roofline    the render kernel against its binding ceiling.  The bound and its fraction come from
              the rocprofv3 PMC record of this exact library build and config (profiles/
              pmc_records.json, tools/pmc.sh + tools/pmc_summary.py): VALU issue (f64-heavy vector
              ALU) vs HBM.  `achieved` = VALU issue cycles per launch (PMC instruction mix x issue
              cost) / the live HIP-event kernel time; `hbm_frac` = PMC HBM bytes / kernel time / 8 TB/s;
              SURVEY.md 8(d)'s algorithmic-bytes formula is kept as `algorithmic_*` (its bytes are
              served by L2 / MALL, not HBM, so its fraction is no physical bound);
  drop_in     the reference's own call pattern (src/main.rs:197-216): host threads each calling
              vr_partial_render_scene for 1-spp full frames into host AccumulationBuffers, merged
              by vr_merge_tile on the main thread (N = 1, rank 0);
  cpu_baseline the oracle's reference-mode restatement (exhaustive BVH traversal, recursive
              integrator) on the host cores of this box: whole 1-spp passes of the same frame until
              --cpu-seconds have elapsed (N = 1, rank 0).
"""
import argparse
import hashlib
import json
import os
import queue
import sys
import threading
import time

import torch  # import first: the HIP library then binds to torch's HIP runtime (same soname)
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from vanrijn_amd import distributed as D  # noqa: E402
from vanrijn_amd import scenes  # noqa: E402
from vanrijn_amd.render import (AccumulationBuffer, Tile, partial_render_scene, render_tile_device,  # noqa: E402
                                stream_check_error)

METRIC = "Msamples/s + achieved HBM GB/s, 1024x1024 bunny @256spp, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec
SIMDS = 1024            # 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4         # max engine clock (spec)
SEED = 0x5EED0001

# BASELINE.json configs; spp is per frame; `split` spreads it over the ranks
CONFIGS = {
    "c1": dict(scene="bench", width=256, height=256, spp=16, split=False),
    "c2": dict(scene="main", width=512, height=512, spp=64, split=False),
    "c3": dict(scene="main", width=1024, height=1024, spp=256, split=False),
    "c4": dict(scene="main", width=2048, height=2048, spp=1024, split=True),
    "c5": dict(scene="c5", width=4096, height=4096, spp=256, split=True),
}

# SURVEY.md 8(d)'s algorithmic bytes, per-unit figures as written: one f64 AABB (48 B) per box
# test, a triangle's 9 f64 vertices (72 B) per triangle test, its 9 f64 normals (72 B) per shaded
# triangle hit, one f64 (X, Y, Z, W) record (32 B) per pixel.
BYTES_PER_BOX_TEST = 48
BYTES_PER_TRI_TEST = 72
BYTES_PER_SHADED_TRI = 72
BYTES_PER_PIXEL_STATE = 32

# Issue cost of one wave64 VALU instruction on a gfx950 SIMD, in cycles (MI355X_MICROARCH.md:
# wave64 f32 VALU over 2 cycles; f64 FMA/ADD/MUL at half the f32 rate (78.6 vs 157.3 TF spec);
# f64 transcendentals (rcp/rsq/sqrt) taken at a quarter of the f64 rate).  Other f64 opcodes
# (div_scale/fmas/fixup, compares, min/max) are counted at the f32 cost: a lower bound.
VALU_CYCLES = {"other": 2, "f64": 4, "trans_f64": 16}


def algorithmic_bytes(c, pixels):
    return (BYTES_PER_BOX_TEST * c["box_tests"] + BYTES_PER_TRI_TEST * c["triangle_tests"] +
            BYTES_PER_SHADED_TRI * c["shaded_triangle_hits"] + BYTES_PER_PIXEL_STATE * pixels)


def layout_bytes(c, pixels):
    """What this kernel's own layout reads and writes per launch before any cache: a 128-B Node4
    line per wide-node visit, a 48-B f64 box per exact fallback, the 80-B vertex record per triangle
    test, vertex + normal records (160 B) per shaded triangle hit, the 16-B staged photon per sample,
    the 64-B accumulation record per pixel."""
    return (128 * c["node_visits"] + 48 * c["exact_box_tests"] + 80 * c["triangle_tests"] +
            160 * c["shaded_triangle_hits"] + 16 * c["samples"] + 64 * pixels)


def config_key(scene, width, height, spp):
    return f"{scene} {width}x{height} spp{spp}"


def lib_sha():
    from vanrijn_amd import _native as N
    return hashlib.sha256(open(N.LIB_PATH, "rb").read()).hexdigest()


def pmc_record(key):
    """The committed PMC record of this library build on this config, or None."""
    try:
        recs = json.load(open(os.path.join(ROOT, "profiles", "pmc_records.json")))
    except (OSError, ValueError):
        return None
    rec = recs.get(key)
    if not rec or rec.get("lib_sha256") != lib_sha():
        return None
    return rec


def valu_issue_cycles(pmc):
    f64 = pmc["SQ_INSTS_VALU_FMA_F64"] + pmc["SQ_INSTS_VALU_ADD_F64"] + pmc["SQ_INSTS_VALU_MUL_F64"]
    trans = pmc["SQ_INSTS_VALU_TRANS_F64"]
    other = pmc["SQ_INSTS_VALU"] - f64 - trans
    return VALU_CYCLES["other"] * other + VALU_CYCLES["f64"] * f64 + VALU_CYCLES["trans_f64"] * trans


def roofline(counts, pixels, kernel_s, key, passes=1):
    """kernel_s: the render kernel's time per step (all its launches: a frame whose staging exceeds
    the per-launch cap runs in `passes` equal launches); the PMC record holds one launch, so its
    rates use the per-launch time kernel_s / passes."""
    alg = algorithmic_bytes(counts, pixels)
    r = {"kernel": "render_kernel", "kernel_ms": round(kernel_s * 1e3, 3), "launches_per_step": passes,
         "algorithmic_bytes_per_launch": alg,
         "algorithmic_gbs": round(alg / kernel_s / 1e9, 2),
         "algorithmic_frac": round(alg / kernel_s / 1e9 / HBM_PEAK_GBS, 4),
         "layout_bytes_per_launch": layout_bytes(counts, pixels),
         "layout_gbs": round(layout_bytes(counts, pixels) / kernel_s / 1e9, 2),
         "counters_per_launch": {k: counts[k] for k in ("box_tests", "node_visits", "triangle_tests", "rays",
                                                        "shaded_triangle_hits", "samples", "traversal_slots",
                                                        "path_loop_slots", "exact_box_tests")},
         "traversal_lane_utilisation": round(counts["node_visits"] / max(1, counts["traversal_slots"]), 4),
         "path_loop_lane_utilisation": round(counts["rays"] / max(1, counts["path_loop_slots"]), 4)}
    rec = pmc_record(key)
    if rec is None:
        r.update({"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None,
                  "pmc": f"no PMC record for this library build on '{key}' (tools/pmc.sh)"})
        return r
    pmc = rec["per_launch"]
    launch_s = kernel_s / max(1, passes)
    traffic = 2 * pmc["FETCH_SIZE"] * 1024 + pmc["WRITE_SIZE"] * 1024  # gfx950: FETCH_SIZE counts 128-B lines at 64 B
    hbm_gbs = traffic / launch_s / 1e9
    valu = valu_issue_cycles(pmc)
    valu_rate = valu / launch_s / 1e9  # G SIMD-cycles of VALU issue per second
    valu_peak = SIMDS * CLOCK_GHZ
    clk = pmc["GRBM_GUI_ACTIVE"] / 8 / (rec["kernel_ns"] * 1e-9) / 1e9  # effective clock of the profiled launch
    fracs = {"valu": valu_rate / valu_peak, "hbm": hbm_gbs / HBM_PEAK_GBS}
    bound = max(fracs, key=fracs.get)
    r.update({
        "bound": bound,
        "achieved": round(valu_rate, 2) if bound == "valu" else round(hbm_gbs, 2),
        "peak": valu_peak if bound == "valu" else HBM_PEAK_GBS,
        "unit": "G VALU issue-cycles/s" if bound == "valu" else "GB/s",
        "frac": round(fracs[bound], 4),
        "traffic": traffic,
        "hbm_gbs": round(hbm_gbs, 2), "hbm_frac": round(fracs["hbm"], 4),
        "valu_issue_frac": round(fracs["valu"], 4),
        "valu_issue_cycles_per_launch": valu, "valu_cost_model_cycles": VALU_CYCLES,
        "valu_insts_per_launch": pmc["SQ_INSTS_VALU"],
        "f64_insts_per_launch": pmc["SQ_INSTS_VALU_FMA_F64"] + pmc["SQ_INSTS_VALU_ADD_F64"] +
        pmc["SQ_INSTS_VALU_MUL_F64"] + pmc["SQ_INSTS_VALU_TRANS_F64"],
        # rocprof's gfx94x VALUBusy formula (ACTIVE_INST_VALU quad-cycles x 4 / SIMDs / cycles): it sums
        # per-wave busy time, so waves interleaving on one SIMD count twice -- an upper bound
        "valu_busy_pmc": round(pmc["SQ_ACTIVE_INST_VALU"] * 4 / SIMDS / (pmc["GRBM_GUI_ACTIVE"] / 8), 4),
        "wave_wait_any_frac": round(pmc["SQ_WAIT_ANY"] / pmc["SQ_WAVE_CYCLES"], 4),
        "l2_hit_rate": round(pmc["TCC_HIT_sum"] / (pmc["TCC_HIT_sum"] + pmc["TCC_MISS_sum"]), 4)
        if "TCC_HIT_sum" in pmc else None,
        "profiled_clock_ghz": round(clk, 3),
        "pmc": rec.get("source"),
    })
    return r


# ---------------------------------------------------------------------------- host / CPU baseline
def cpu_info():
    """Cores this process may use: the affinity mask, capped by a cgroup CPU quota if any."""
    affinity = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            quota = q / p if q > 0 else None
        except (OSError, ValueError):
            pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = affinity if quota is None else max(1, min(affinity, int(quota)))
    return {"nproc": os.cpu_count(), "affinity": affinity, "cgroup_quota_cpus": quota, "usable": usable,
            "model": model}


def cpu_baseline(scene, width, height, seconds, threads):
    """Oracle (reference mode) on the host: 1-spp passes of the frame (a central band of about 1M
    pixels for frames above 1024^2), sample indices 0, 1, 2, ... until `seconds` have elapsed (at
    least 2 passes); every pass is timed, so the spread is reported."""
    from oracle import oracle_ffi as O
    orc = O.OracleScene(scene.spec())
    band = max(1, min(height, (1 << 20) // width))
    r0 = (height - band) // 2
    t = Tile(0, width, r0, r0 + band)
    rates, total_t, samples, k = [], 0.0, 0, 0
    while k < 2 or total_t < seconds:
        t0 = time.perf_counter()
        orc.render_tile(t, height, width, 1, SEED, k, O.MODE_REFERENCE, threads)
        dt = time.perf_counter() - t0
        n = t.width() * t.height()
        rates.append(n / dt / 1e6)
        total_t += dt
        samples += n
        k += 1
    where = "full frame" if band == height else f"rows {r0}..{r0 + band - 1} of the frame"
    return {"value": round(samples / total_t / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "per_pass_msamples_s": {"min": round(min(rates), 4), "max": round(max(rates), 4),
                                    "passes": len(rates)},
            "sample": f"{width}x{height} image, {where}, {k} 1-spp passes (sample indices 0..{k - 1}, "
                      f"{samples} samples, {total_t:.1f} s), oracle reference mode (exhaustive line-BVH "
                      f"traversal, recursive integrator), {threads} threads"}


def drop_in_leg(dscene, width, height, frames, threads, device):
    """src/main.rs:197-216 through the C ABI: `threads` workers each call partial_render_scene
    (1 spp, whole frame, host AccumulationBuffer) until `frames` passes are done; the main thread
    merges every returned buffer into the image with merge_tile."""
    tile = Tile(0, width, 0, height)
    image = AccumulationBuffer(width, height)
    partial_render_scene(dscene, tile, height, width, device=device)  # warm the call contexts
    q = queue.Queue(maxsize=2 * threads)
    todo = iter(range(frames))
    lock = threading.Lock()

    def worker():
        while True:
            with lock:
                if next(todo, None) is None:
                    break
            q.put(partial_render_scene(dscene, tile, height, width, device=device))
        q.put(None)

    t0 = time.perf_counter()
    ws = [threading.Thread(target=worker) for _ in range(threads)]
    for w in ws:
        w.start()
    live, merged = threads, 0
    while live:
        b = q.get()
        if b is None:
            live -= 1
            continue
        image.merge_tile(tile, b)
        merged += 1
    dt = time.perf_counter() - t0
    for w in ws:
        w.join()
    assert merged == frames and float(image.weight_buffer.min()) == frames
    return {"value": round(frames * width * height / dt / 1e6, 3), "unit": "Msamples/s", "threads": threads,
            "frames": frames, "ms_per_frame": round(dt / frames * 1e3, 3),
            "pattern": "main.rs:197-216: worker threads x vr_partial_render_scene (1 spp, full frame, host "
                       "buffers: 88 B/pixel back over PCIe), vr_merge_tile on the main thread"}


# ---------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c3",
                    help="BASELINE.json configs (SURVEY.md 8(d)); c4 / c5 split one frame's spp over the ranks")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None, help="per frame (split over ranks for c4 / c5)")
    ap.add_argument("--scene", choices=["main", "bench", "c5"], default=None,
                    help="main: main.rs scene; bench: benches/simple_scene.rs; "
                         "c5: main.rs's plane and spheres + the 1,051,392-triangle synthetic mesh")
    ap.add_argument("--mesh", default=None,
                    help="the reference's test_data/stanford_bunny.obj (size + sha256 verified) instead of the "
                         "procedural stand-in")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=None, help="default: every core this process may use")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--drop-in-frames", type=int, default=64)
    ap.add_argument("--drop-in-threads", type=int, default=8)
    ap.add_argument("--no-drop-in", action="store_true")
    args = ap.parse_args()

    cfg = dict(CONFIGS[args.config])
    for k in ("width", "height", "spp", "scene"):
        if getattr(args, k) is not None:
            cfg[k] = getattr(args, k)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    torch.cuda.set_device(local)
    # launched by torch.distributed.run (RANK set): the RCCL group is created even at world size 1,
    # so a one-GPU box rehearses the multi-GPU step (init, barriers, reduce, max-over-ranks timing)
    distributed = world > 1 or "RANK" in os.environ
    if distributed:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    W, H = cfg["width"], cfg["height"]
    spp = D.shard_spp(cfg["spp"], world, cfg["split"])  # this rank's samples per pixel per frame
    if cfg["scene"] == "c5":
        scene = scenes.synthetic_scene()
    else:
        scene = scenes.main_scene(args.mesh) if cfg["scene"] == "main" else scenes.bench_scene(args.mesh)
    dscene = scene.device_scene(local)
    info = dscene.info()
    tile = Tile(0, W, 0, H)
    state = torch.zeros(H * W * 8, dtype=torch.float64, device=f"cuda:{local}")
    stream = torch.cuda.current_stream()

    def step(i, timed=False):
        def shard(first, st):
            return render_tile_device(dscene, tile, H, W, spp, SEED, first, st.data_ptr(), stream.cuda_stream,
                                      timed=timed, device=local)
        return D.frame_step(shard, state, i, spp)

    # counting launch (untimed): traversal counters of exactly this workload
    counts = render_tile_device(dscene, tile, H, W, spp, SEED, rank * spp, state.data_ptr(), stream.cuda_stream,
                                counters=True, device=local)
    for i in range(args.warmup):
        step(1 + i)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    kernel_ms, reduce_ms, passes = [], [], []
    t0 = time.perf_counter()
    for i in range(args.steps):
        st = step(1 + args.warmup + i, timed=True)
        kernel_ms.append(st["kernel_ms"])  # render kernel only (HIP events on the launch stream)
        reduce_ms.append(st["reduce_ms"])  # the ordered per-pixel Kahan reduce after it
        passes.append(int(st.get("passes", 1)) or 1)  # launches per frame (staging cap)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    stream_check_error(dscene, stream.cuda_stream, device=local)  # device errors of the untimed steps
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    samples = world * args.steps * W * H * spp
    value = samples / elapsed / 1e6
    avg_kernel_s = sum(kernel_ms) / len(kernel_ms) / 1e3
    workload = {"main": f"main.rs scene (plane, 3 spheres, Lambertian bunny), {W}x{H}",
                "bench": f"bench scene (reflective bunny), {W}x{H}",
                "c5": f"C5: main.rs plane + spheres + 1,051,392-triangle synthetic mesh, {W}x{H}"}[cfg["scene"]]
    workload += (f" @{cfg['spp']}spp per frame split over {world} GPU(s) ({spp} each)" if cfg["split"]
                 else f" @{spp}spp per GPU")
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong" if cfg["split"] else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic: lat-long displaced sphere mesh (1,051,392 triangles, seed 0x1DEA), counter-based RNG "
                 "seed 0x5EED0001") if cfg["scene"] == "c5" else
                ("synthetic: procedural bunny stand-in (69,312 triangles; the reference OBJ is an LFS pointer), "
                 "counter-based RNG seed 0x5EED0001") if args.mesh is None else
                f"{os.path.basename(args.mesh)} (sha256-verified reference bunny), counter-based RNG seed 0x5EED0001",
        "config": {"workload": workload, "config": args.config, "width": W, "height": H, "spp_per_gpu": spp,
                   "triangles": info["triangle_count"], "bvh_depth": info["max_bvh_depth"],
                   "parallelism": f"spp-split x{world}, RCCL reduce",
                   "pmc_key": config_key(cfg["scene"], W, H, spp)},
        "roofline": roofline(counts, W * H, avg_kernel_s, config_key(cfg["scene"], W, H, spp), max(passes)),
    }
    out["roofline"]["reduce_kernel_ms"] = round(sum(reduce_ms) / len(reduce_ms), 3)
    # samples of 8x8 blocks whose camera rays all miss every object (block_cull_kernel) are applied
    # as the photon {0, 0} without tracing: the records are bit-identical with VR_BLOCK_CULL=0
    # (tests/test_gpu_cull.py); every sample is counted in `value`
    out["roofline"]["frustum_culled_sample_fraction"] = round(1.0 - counts["samples"] / (W * H * spp), 4)
    if rank == 0 and world == 1 and not args.no_drop_in:
        out["drop_in"] = drop_in_leg(dscene, W, H, args.drop_in_frames, args.drop_in_threads, local)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        ci = cpu_info()
        threads = args.cpu_threads or ci["usable"]
        out["cpu_baseline"] = cpu_baseline(scene, W, H, args.cpu_seconds, threads)
        out["cpu_baseline"]["host"] = ci
    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

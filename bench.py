#!/usr/bin/env python3
"""Benchmark: Msamples/s of the MI355X path-tracing core on BASELINE.json's headline config.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1|c2|c3|c4|c5]

--gpus N > 1 runs N ranks, one process per GPU: under `python -m torch.distributed.run
--nproc-per-node N ... bench.py --gpus N ...` (the driver's launch) the ranks come from the
environment; started directly, bench.py starts that launcher itself as ONE child process tree before
anything touches the GPU (launch_ranks: never a re-exec), waits for it and forwards rank 0's JSON line.
A WORLD_SIZE other than --gpus, or fewer GPUs on the node than --gpus, is an error (exit status 2),
never a silent smaller run; `n_gpus` is the process group's dist.get_world_size().

Workload (default --config c3 = BASELINE.json configs[2] / metric): the main.rs scene
(src/main.rs:120-189: plane, three spheres, Lambertian bunny; camera (-2, 1, -5)) at 1024x1024,
256 samples per pixel per GPU.  The bunny OBJ is a Git-LFS pointer in the reference, so the mesh is
the deterministic procedural stand-in (69,312 triangles, vanrijn_amd/scenes.py).  One "step" = one
frame: rank r renders sample indices [(step*N + r)*spp, +spp) of the same image -- c3, c4 and c5
split ONE frame's 256 / 1024 / 256 spp over the N ranks (strong scaling: the metric's "1024x1024
@256spp, 1/2/4/8 GPUs" is a fixed workload), c1 / c2 give every rank a whole frame (weak) -- then the
per-pixel sums {X, Y, Z, weight} (32 B) are summed onto rank 0 with one RCCL reduce over xGMI inside
the timed region (vanrijn_amd/distributed.py frame_step, the same step the gloo tests run).  At N > 1
a split config also times every rank rendering the whole frame (`weak_scaling`, secondary), and rank 0
runs the PMC passes on its own shard after the timed regions (`roofline`).

Printed (rank 0, one JSON line):
  value       total samples of all ranks / max-over-ranks wall time of the timed steps;
  roofline    the render kernel against its binding ceiling, from rocprofv3 PMC passes run by this
              bench itself on this build and workload (live_pmc: child processes, one counter group
              each; the committed profiles/pmc_records.json only if they fail): VALU issue (f64-heavy
              vector ALU) vs HBM.  `achieved` = the SIMD-cycles the hardware spent issuing VALU per
              launch (4 x SQ_ACTIVE_INST_VALU) / the live HIP-event kernel time, `peak` = 1024 SIMDs
              x 2.4 GHz, `frac` = achieved / peak (measured, not priced); `useful_lane_frac` = frac x
              the lane efficiency of what was issued; `valu_issue_frac_model` prices the PMC
              instruction mix at the per-class issue costs tools/opcost.hip measured (profiles/r03/
              opcost.json); `hbm_frac` = PMC HBM bytes (2 FETCH_SIZE + WRITE_SIZE) / kernel time /
              8 TB/s; SURVEY.md 8(d)'s algorithmic-bytes formula is kept as `cache_served_*` (its
              bytes are served by L2 / MALL, not HBM, so its fraction is no bound -- above 1 at C3);
              lane utilisation and per-launch counters come from a counting launch of the same
              workload and need no PMC;
  traced_msamples_per_s  the samples actually traced per second (`value` also counts the samples of
              frustum-culled 8x8 blocks, applied in closed form: `frustum_culled_sample_fraction`);
  scene_build vr_scene_create time (excluded from `value`);
  reduce      bytes and RCCL time per step of the cross-GPU reduce;
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
from vanrijn_amd.render import (AccumulationBuffer, Tile, collect_launch_times, partial_render_scene,  # noqa: E402
                                render_tile_device, stream_check_error)

METRIC = "Msamples/s + achieved HBM GB/s, 1024x1024 bunny @256spp, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec
SIMDS = 1024            # 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4         # max engine clock (spec)
SEED = 0x5EED0001

# BASELINE.json configs; spp is per frame; `split` spreads it over the ranks
CONFIGS = {
    "c1": dict(scene="bench", width=256, height=256, spp=16, split=False),
    "c2": dict(scene="main", width=512, height=512, spp=64, split=False),
    # the metric's own workload: ONE 1024^2 @256spp frame, its samples split over the 1/2/4/8 GPUs
    # (strong scaling; the weak figure -- every rank a whole frame -- is the line's `weak_scaling`)
    "c3": dict(scene="main", width=1024, height=1024, spp=256, split=True),
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

# Issue cost of one wave64 VALU instruction on a gfx950 SIMD, in cycles, MEASURED by
# tools/opcost.hip (profiles/r03/opcost.json): SIMD busy cycles per instruction with 3 waves per
# SIMD -- the render kernel's occupancy -- each issuing independent instructions of one opcode.
# Every rocprofv3 instruction class is priced by its representative opcodes; the remainder of
# SQ_INSTS_VALU (moves, selects, compares, logic, bit-field ops) by the median of those opcodes.
OPCOST_PATH = os.path.join(ROOT, "profiles", "r03", "opcost.json")
OCCUPANCY_WAVES_PER_SIMD = 3
PMC_CLASS_OPCODES = {
    "SQ_INSTS_VALU_FMA_F64": ["v_fma_f64", "v_div_fmas_f64"],
    "SQ_INSTS_VALU_ADD_F64": ["v_add_f64"],
    "SQ_INSTS_VALU_MUL_F64": ["v_mul_f64"],
    "SQ_INSTS_VALU_TRANS_F64": ["v_rcp_f64", "v_sqrt_f64", "v_rsq_f64"],
    "SQ_INSTS_VALU_INT64": ["v_lshlrev_b64", "v_mad_u64_u32"],
    "SQ_INSTS_VALU_INT32": ["v_add_u32", "v_mul_lo_u32", "v_bfe_u32"],
    "SQ_INSTS_VALU_FMA_F32": ["v_fma_f32", "v_pk_fma_f32"],
    "SQ_INSTS_VALU_ADD_F32": ["v_add_f32"],
    "SQ_INSTS_VALU_MUL_F32": ["v_mul_f32"],
    "SQ_INSTS_VALU_TRANS_F32": None,  # not measured: MI355X_MICROARCH.md's 8 cycles (v_exp_f32 ...)
    "SQ_INSTS_VALU_CVT": ["v_cvt_f64_i32", "v_cvt_f32_f64"],
}
OTHER_OPCODES = ["v_mov_b32", "v_xor_b32", "v_cndmask_b32_e64 (sgpr mask)", "v_cmp_lt_f32", "v_cmp_lt_u32",
                 "v_cmp_lt_f64", "v_max_f32", "v_max_f64", "v_min_f64", "v_div_scale_f64", "v_div_fixup_f64"]


def progress(msg):
    """A progress line on stderr (a long run shows it is alive; stdout carries only the JSON line)."""
    print(f"bench.py [{time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def issue_costs():
    """Cycles per instruction per PMC class from the committed microbenchmark (None if absent)."""
    try:
        rows = json.load(open(OPCOST_PATH))["results"]
    except (OSError, ValueError, KeyError):
        return None
    cpi = {r["op"]: r["cycles_per_inst"] for r in rows if r["waves_per_simd"] == OCCUPANCY_WAVES_PER_SIMD}

    def mean(ops):
        v = [cpi[o] for o in ops if o in cpi]
        return sum(v) / len(v) if v else None

    other = sorted(cpi[o] for o in OTHER_OPCODES if o in cpi)
    if not other:
        return None
    costs = {"other": other[len(other) // 2]}
    for k, v in PMC_CLASS_OPCODES.items():
        # a class without a measured opcode: TRANS_F32 at the guide's 8 cycles, else "other"
        costs[k] = (mean(v) if v else None) or (8.0 if v is None else costs["other"])
    return costs


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


def valu_issue_cycles(pmc, costs):
    classified = sum(pmc[k] for k in PMC_CLASS_OPCODES)
    return sum(pmc[k] * costs[k] for k in PMC_CLASS_OPCODES) + (pmc["SQ_INSTS_VALU"] - classified) * costs["other"]


# ---------------------------------------------------------------------------- live PMC (rocprofv3)
# One counter group per rocprofv3 run, --kernel-trace beside --pmc only (MI355X_MICROARCH.md), each
# pass a child process (bench.py --pmc-child: the same workload, one timed frame) under its own time
# limit; nothing here runs under the profiler itself.
PMC_PASSES = [
    ("fetch", ["FETCH_SIZE"]),
    ("write", ["WRITE_SIZE"]),
    ("mix1", ["SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
              "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_CVT"]),
    ("mix2", ["SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_TRANS_F32",
              "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_BUSY_CYCLES", "SQ_WAVES"]),
    ("tcc", ["TCC_HIT_sum", "TCC_MISS_sum", "GRBM_GUI_ACTIVE"]),
    # hardware VALU activity and lane use: the cycles waves spend issuing VALU, and
    # the lane-cycles of work they did; with this pass's own clock (GRBM_GUI_ACTIVE, 8 XCDs)
    ("lanes", ["SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE"]),
]
# counters a pass repeats from another, kept under "<name>@<pass>"
PMC_PASS_LOCAL = {"lanes": ("SQ_INSTS_VALU", "GRBM_GUI_ACTIVE")}


def _is_timed_render(name):
    # render_kernel<STACK, COUNT, RECORD, ...>: the timed launches have COUNT = false, RECORD = false
    if "render_kernel<" not in name:
        return False
    targs = name.split("render_kernel<")[1].split(">")[0].split(",")
    return targs[1].strip() == "false" and targs[2].strip() == "false"


def _fold_pass(d):
    import csv
    per, dur = {}, {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if _is_timed_render(r["Kernel_Name"]):
            x = per.setdefault(int(r["Dispatch_Id"]), {})
            x[r["Counter_Name"]] = x.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    tr = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(tr):
        for r in csv.DictReader(open(tr)):
            if _is_timed_render(r["Kernel_Name"]):
                dur[int(r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    last = max(per)
    return per[last], dur.get(last)


def live_pmc(child_args, timeout_s=150):
    """Run the PMC passes on this build and workload; returns a record like profiles/pmc_records.json's
    (per_launch counters, kernel_ns) or {"error": ...}."""
    import shutil
    import signal
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return {"error": "rocprofv3 not found"}
    tmp = tempfile.mkdtemp(prefix="vr_pmc_")
    # a one-process child even under torch.distributed.run (rank 0 at N > 1): no rank variables
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "ROLE_WORLD_SIZE", "GROUP_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
           and not k.startswith("TORCHELASTIC_")}
    env["TMPDIR"] = tmp
    per_launch, kernel_ns = {}, {}
    try:
        for name, counters in PMC_PASSES:
            d = os.path.join(tmp, name)
            cmd = [prof, "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run", "--pmc"] + counters + \
                  ["--", sys.executable, os.path.abspath(__file__), "--pmc-child"] + child_args
            p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, start_new_session=True,
                                 env=env)
            try:
                rc = p.wait(timeout=timeout_s)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
                return {"error": f"PMC pass {name} exceeded {timeout_s} s"}
            if rc != 0:
                return {"error": f"PMC pass {name} exited {rc}"}
            c, ns = _fold_pass(d)
            progress(f"PMC pass {name}: {', '.join(counters)}")
            for k in PMC_PASS_LOCAL.get(name, ()):
                if k in c:
                    c[f"{k}@{name}"] = c.pop(k)
            per_launch.update(c)
            if ns:
                kernel_ns[name] = ns
    except (OSError, ValueError, KeyError) as e:
        return {"error": f"PMC passes: {e}"}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return {"per_launch": per_launch, "kernel_ns": kernel_ns.get("tcc") or max(kernel_ns.values()),
            "kernel_ns_per_pass": kernel_ns, "lib_sha256": lib_sha(),
            "source": "live: rocprofv3 --pmc passes of this run's build and workload (bench.py live_pmc)"}


def roofline(counts, pixels, kernel_s, key, passes=1, pmc=None):
    """kernel_s: the render kernel's time per step (all its launches: a frame whose staging exceeds
    the per-launch cap runs in `passes` equal launches); the PMC record holds one launch, so its
    rates use the per-launch time kernel_s / passes.  `pmc`: this run's live PMC record, else the
    committed record of this library build (profiles/pmc_records.json)."""
    alg = algorithmic_bytes(counts, pixels)
    # SURVEY.md 8(d)'s per-unit bytes x this launch's counts: served by L2 and the Infinity Cache
    # (L2 hit rate 0.86 at C3), so their rate is no HBM bound -- it exceeds the HBM peak at C3
    r = {"kernel": "render_kernel", "kernel_ms": round(kernel_s * 1e3, 3), "launches_per_step": passes,
         "cache_served_algorithmic_bytes_per_launch": alg,
         "cache_served_algorithmic_gbs": round(alg / kernel_s / 1e9, 2),
         "cache_served_algorithmic_frac_of_hbm_peak": round(alg / kernel_s / 1e9 / HBM_PEAK_GBS, 4),
         "layout_bytes_per_launch": layout_bytes(counts, pixels),
         "layout_gbs": round(layout_bytes(counts, pixels) / kernel_s / 1e9, 2),
         "counters_per_launch": {k: counts[k] for k in ("box_tests", "node_visits", "triangle_tests", "rays",
                                                        "shaded_triangle_hits", "samples", "traversal_slots",
                                                        "path_loop_slots", "exact_box_tests")},
         "traversal_lane_utilisation": round(counts["node_visits"] / max(1, counts["traversal_slots"]), 4),
         "path_loop_lane_utilisation": round(counts["rays"] / max(1, counts["path_loop_slots"]), 4)}
    rec = pmc if pmc and "per_launch" in pmc else pmc_record(key)
    costs = issue_costs()
    if rec is None or costs is None:
        why = (pmc or {}).get("error") or f"no PMC record for this library build on '{key}' (tools/pmc.sh)"
        r.update({"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None,
                  "pmc": why if rec is None else "no opcode cost table (profiles/r03/opcost.json)"})
        return r
    pmc = rec["per_launch"]
    launch_s = kernel_s / max(1, passes)
    traffic = 2 * pmc["FETCH_SIZE"] * 1024 + pmc["WRITE_SIZE"] * 1024  # gfx950: FETCH_SIZE counts 128-B lines at 64 B
    hbm_gbs = traffic / launch_s / 1e9
    valu = valu_issue_cycles(pmc, costs)
    valu_rate = valu / launch_s / 1e9  # G SIMD-cycles of VALU issue per second (priced model)
    valu_peak = SIMDS * CLOCK_GHZ
    clk = pmc["GRBM_GUI_ACTIVE"] / 8 / (rec["kernel_ns"] * 1e-9) / 1e9  # effective clock of the profiled launch
    # measured: the SIMD-cycles the hardware spent issuing VALU (SQ_ACTIVE_INST_VALU
    # counts per SIMD-quad: x4), per second of the live kernel time -- the line's headline fraction
    busy = 4 * pmc["SQ_ACTIVE_INST_VALU"] if pmc.get("SQ_ACTIVE_INST_VALU") else None
    busy_rate = busy / launch_s / 1e9 if busy else None
    lane_eff = pmc["SQ_THREAD_CYCLES_VALU"] / (64 * pmc["SQ_ACTIVE_INST_VALU"]) if busy else None
    fracs = {"valu": (busy_rate if busy else valu_rate) / valu_peak, "hbm": hbm_gbs / HBM_PEAK_GBS}
    bound = max(fracs, key=fracs.get)
    r.update({
        "bound": bound,
        "achieved": round(busy_rate if busy else valu_rate, 2) if bound == "valu" else round(hbm_gbs, 2),
        "peak": valu_peak if bound == "valu" else HBM_PEAK_GBS,
        "unit": ("G VALU-busy SIMD-cycles/s" if busy else "G VALU issue-cycles/s (priced)") if bound == "valu"
        else "GB/s",
        "frac": round(fracs[bound], 4),
        "frac_source": "hardware: 4 SQ_ACTIVE_INST_VALU / live kernel time / (1024 SIMDs x 2.4 GHz)" if busy
        else "priced model (SQ_ACTIVE_INST_VALU not collected)",
        "useful_lane_frac": round(fracs["valu"] * lane_eff, 4) if busy else None,
        "traffic": traffic,
        "hbm_gbs": round(hbm_gbs, 2), "hbm_frac": round(fracs["hbm"], 4),
        "valu_issue_frac_model": round(valu_rate / valu_peak, 4),
        # the priced issue cycles against the profiled launch's own clock (DVFS holds it below 2.4 GHz)
        "valu_issue_frac_model_at_profiled_clock": round(valu / (rec["kernel_ns"] * 1e-9) / (SIMDS * clk * 1e9), 4),
        "valu_issue_cycles_per_launch": valu,
        "valu_cost_model_cycles": {k: round(v, 3) for k, v in costs.items()},
        "valu_cost_source": os.path.relpath(OPCOST_PATH, ROOT) + " (tools/opcost.hip, 3 waves/SIMD)",
        "valu_insts_per_launch": pmc["SQ_INSTS_VALU"],
        "f64_insts_per_launch": pmc["SQ_INSTS_VALU_FMA_F64"] + pmc["SQ_INSTS_VALU_ADD_F64"] +
        pmc["SQ_INSTS_VALU_MUL_F64"] + pmc["SQ_INSTS_VALU_TRANS_F64"],
        "wave_wait_any_frac": round(pmc["SQ_WAIT_ANY"] / pmc["SQ_WAVE_CYCLES"], 4)
        if pmc.get("SQ_WAVE_CYCLES") else None,
        "l2_hit_rate": round(pmc["TCC_HIT_sum"] / (pmc["TCC_HIT_sum"] + pmc["TCC_MISS_sum"]), 4)
        if "TCC_HIT_sum" in pmc else None,
        # measured, not priced: 4 SQ_ACTIVE_INST_VALU per SIMD-cycle of the profiled
        # launch (GRBM_GUI_ACTIVE / 8 XCDs) -- the VALU-busy fraction of all 1024 SIMDs -- and the lane
        # efficiency of what was issued, SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU)
        "valu_active_frac": round(4 * pmc["SQ_ACTIVE_INST_VALU"] / (SIMDS * pmc["GRBM_GUI_ACTIVE@lanes"] / 8), 4)
        if pmc.get("GRBM_GUI_ACTIVE@lanes") else None,
        "valu_lane_efficiency": round(pmc["SQ_THREAD_CYCLES_VALU"] / (64 * pmc["SQ_ACTIVE_INST_VALU"]), 4)
        if pmc.get("SQ_ACTIVE_INST_VALU") else None,
        "profiled_clock_ghz": round(clk, 3),
        "profiled_kernel_ms": round(rec["kernel_ns"] / 1e6, 3),
        "pmc": rec.get("source"),
        "pmc_per_launch": {k: pmc[k] for k in sorted(pmc)},
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
    # warm-up: one call per worker at once, so the `threads` call contexts (stream, staging, page-
    # locked host buffer: ~150 MB of allocations each at 1024^2) exist before the timed frames, as
    # they do in main.rs's steady state; one warm call warmed a single context and the other seven
    # were created inside the timed region
    warm = [threading.Thread(target=partial_render_scene, args=(dscene, tile, height, width),
                             kwargs={"device": device}) for _ in range(threads)]
    for w in warm:
        w.start()
    for w in warm:
        w.join()
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
            "pattern": "main.rs:197-216: worker threads x vr_partial_render_scene (1 spp, full frame into a "
                       "fresh host buffer: only colour_sum, 24 B/pixel, crosses PCIe; the host derives the "
                       "other 64 B/pixel of the 88-B AccumulationBuffer layout), vr_merge_tile on the main thread"}


# ---------------------------------------------------------------------------- rank launcher
def launch_ranks(argv, n, stub=False):
    """`--gpus n` (n > 1) started without torch.distributed.run's environment: start
    `python -m torch.distributed.run --nproc-per-node n ... bench.py <argv>` as one child process tree
    (one fresh process per GPU: this process has not touched the GPU -- torch.cuda.device_count()
    does not initialise it on this image -- and it is never replaced by exec), wait, and forward the
    JSON line rank 0 prints.  Returns the exit status.  `stub`: the CPU test of this launcher (gloo
    ranks, tests/test_bench_launcher.py), no GPU count check."""
    import socket
    import subprocess
    if not stub:
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py: --gpus {n} needs {n} GPUs on this node, found {have}; refusing to report a "
                  f"{have}-GPU run as {n}", file=sys.stderr, flush=True)
            return 2
    with socket.socket() as sk:  # a free rendezvous port on the loopback address
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    print("bench.py: starting " + " ".join(cmd[1:]), file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    lines = []
    for line in p.stdout:  # rank 0's JSON line; anything else goes to stderr
        if line.lstrip().startswith("{"):
            lines.append(line.strip())
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    rc = p.wait()
    if rc == 0 and len(lines) != 1:
        print(f"bench.py: expected one JSON line from rank 0, got {len(lines)}", file=sys.stderr, flush=True)
        return 1
    for line in lines:
        print(line, flush=True)
    return rc


def stub_rank_body():
    """A rank body without the GPU (launcher test): a gloo group, each rank's view of its launch
    environment gathered on rank 0, which prints one JSON line."""
    dist.init_process_group("gloo")
    mine = {k: int(os.environ[k]) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    mine["pid"] = os.getpid()
    got = [None] * dist.get_world_size()
    dist.all_gather_object(got, mine)
    if dist.get_rank() == 0:
        print(json.dumps({"stub": True, "n_gpus": dist.get_world_size(), "ranks": got}), flush=True)
    dist.destroy_process_group()


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
    ap.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 PMC passes of the roofline")
    ap.add_argument("--streams", type=int, default=None,
                    help="frames alternate over this many streams / record buffers (2: a frame's render "
                         "overlaps the previous frame's launch tail, ordered reduce and collective); "
                         "default 1 on one GPU, 2 at N > 1")
    ap.add_argument("--host-build", action="store_true",
                    help="render the host-built traversal tree instead of the device-built one (same images)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)  # one profiled frame (live_pmc)
    ap.add_argument("--stub-ranks", action="store_true", help=argparse.SUPPRESS)  # launcher test (CPU, gloo)
    # tests/test_gpu_dist_rehearsal.py: N ranks on ONE GPU (gloo, the collective on host copies of the
    # sums) -- every step of the N-rank path but the RCCL transport, on a one-GPU box
    ap.add_argument("--one-gpu-rehearsal", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "RANK" not in os.environ and args.gpus > 1:  # start the ranks (nothing has touched the GPU yet)
        return launch_ranks(sys.argv[1:], args.gpus, stub=args.stub_ranks or args.one_gpu_rehearsal)
    if "RANK" in os.environ and int(os.environ.get("WORLD_SIZE", 1)) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {os.environ.get('WORLD_SIZE')}: refusing to run a "
              f"different number of ranks than asked for", file=sys.stderr, flush=True)
        return 2
    if args.stub_ranks:
        stub_rank_body()
        return 0
    if args.pmc_child:
        args.steps, args.warmup, args.no_drop_in, args.no_cpu_baseline, args.no_pmc = 1, 0, True, True, True

    cfg = dict(CONFIGS[args.config])
    for k in ("width", "height", "spp", "scene"):
        if getattr(args, k) is not None:
            cfg[k] = getattr(args, k)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = 0 if args.one_gpu_rehearsal else int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    # launched by torch.distributed.run (RANK set): the RCCL group is created even at world size 1,
    # so a one-GPU box rehearses the multi-GPU step (init, barriers, reduce, max-over-ranks timing)
    distributed = world > 1 or "RANK" in os.environ
    if distributed:
        # a generous timeout: the other ranks wait in the final barrier while rank 0 runs its PMC passes
        import datetime
        if args.one_gpu_rehearsal:
            dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=30))
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                    timeout=datetime.timedelta(minutes=30))
        world = dist.get_world_size()  # what the line reports as n_gpus
        assert world == args.gpus, (world, args.gpus)

    W, H = cfg["width"], cfg["height"]
    spp = D.shard_spp(cfg["spp"], world, cfg["split"])  # this rank's samples per pixel per frame
    if cfg["scene"] == "c5":
        scene = scenes.synthetic_scene()
    else:
        scene = scenes.main_scene(args.mesh) if cfg["scene"] == "main" else scenes.bench_scene(args.mesh)
    # scene build (excluded from the metric, reported separately): vr_scene_create
    # with the traversal tree built on the device (VR_SCENE_DEVICE_SAH: the reference's median-split
    # tree for the tie ranks, the binned-SAH traversal tree over them, the 4-wide collapse) -- the
    # scene every timed step renders; and, for comparison, the same scene built on the host
    torch.cuda.synchronize()
    t_build = time.perf_counter()
    dscene = scene.device_scene(local, device_sah=not args.host_build)
    info = dscene.info()
    build_s = time.perf_counter() - t_build
    build = {"rendered_tree": "host-built" if args.host_build else "device-built (VR_SCENE_DEVICE_SAH)",
             "seconds": round(build_s, 4)}
    if not args.pmc_child:
        t_build = time.perf_counter()
        scene.device_scene(local, device_sah=args.host_build).info()
        build["other_build_seconds"] = round(time.perf_counter() - t_build, 4)
        build["other_build"] = "device-built (VR_SCENE_DEVICE_SAH)" if args.host_build else \
            "host-built (median ranks + binned SAH + 4-wide on the CPU)"
    tile = Tile(0, W, 0, H)
    # frames alternate over `streams` streams, each with its own record buffer (and, inside the
    # library, its own call context): frame i+1's render starts while frame i's launch tail, ordered
    # reduce and cross-GPU collective finish (1: frames strictly one after another)
    # Measured on one MI355X (profiles/r06/probe, r06/small): 1024^2 @32 spp -- the per-rank frame at
    # N = 8 -- 5.95 -> 5.54 ms per frame with 2 streams, C2 (512^2 @64) 3.32 -> 2.88 ms, C1 (256^2 @16,
    # a few trapped mirror paths set a frame's time) 1.64 -> 0.86 ms; @256 spp (c3 at N = 1) 41.18 ->
    # 41.36 ms (no gain): so 2 streams where the ranks' frames are short (<= 64 M samples) or a
    # collective follows each one.  A line with 2 streams also times the frames strictly one after
    # another (`sequential`), so each frame's own latency is reported beside the throughput.
    short = W * H * spp <= (64 << 20)
    nstreams = max(1, args.streams if args.streams else (2 if world > 1 or short else 1))
    states = [torch.zeros(H * W * 8, dtype=torch.float64, device=f"cuda:{local}") for _ in range(nstreams)]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(nstreams - 1)]
    state, stream = states[0], streams[0]

    def step(i, spp_r, timer=None, timed=False, defer=False, ns=None):
        # defer: the render's HIP events are recorded but not waited for (VR_LAUNCH_DEFER_TIMES), so
        # back-to-back timed frames queue without a host round trip between them; their times are
        # collected after the timed region
        j = i % (ns or nstreams)
        st_j = streams[j]

        def shard(first, st):
            return render_tile_device(dscene, tile, H, W, spp_r, SEED, first, st.data_ptr(), st_j.cuda_stream,
                                      timed=timed and not defer, defer_times=defer, device=local)
        with torch.cuda.stream(st_j):  # the collective, the zeroing and the timer events follow the render
            return D.frame_step(shard, states[j], i, spp_r, timer=timer, via_host=args.one_gpu_rehearsal)

    def timed_region(spp_r, first_step, ns=None):
        """args.warmup untimed + args.steps timed frames of spp_r samples per pixel on every rank,
        bracketed by barrier + synchronize; the max over ranks of the wall time, and this rank's
        HIP-event kernel times."""
        for i in range(args.warmup):
            step(first_step + i, spp_r, ns=ns)
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        events = []
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(first_step + args.warmup + i, spp_r, timer=events, defer=True, ns=ns)
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        lt = {"launches": 0, "kernel_ms": 0.0, "reduce_ms": 0.0, "max_passes": 0}
        for st_j in streams:
            stream_check_error(dscene, st_j.cuda_stream, device=local)  # device errors of the untimed steps
            # the timed frames' HIP-event times (render kernel on its launch stream; the ordered
            # per-pixel Kahan reduce after it), and their device errors
            lj = collect_launch_times(dscene, st_j.cuda_stream, device=local)
            for k in ("launches", "kernel_ms", "reduce_ms"):
                lt[k] += lj[k]
            lt["max_passes"] = max(lt["max_passes"], lj["max_passes"])
        assert lt["launches"] == args.steps, lt
        if distributed:
            t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if args.one_gpu_rehearsal else f"cuda:{local}")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return {"elapsed": elapsed, "kernel_s": lt["kernel_ms"] / args.steps / 1e3,
                "reduce_ms": lt["reduce_ms"] / args.steps, "passes": max(1, lt["max_passes"]),
                "rccl_ms": [a.elapsed_time(b) for a, b in events]}

    if args.pmc_child:  # under rocprofv3 (live_pmc): one timed frame of the workload, nothing else
        step(1, spp, timed=True)
        torch.cuda.synchronize()
        return
    progress(f"scene built in {build_s:.3f} s; counting launch")
    # counting launch (untimed): traversal counters of exactly this rank's workload
    counts = render_tile_device(dscene, tile, H, W, spp, SEED, rank * spp, state.data_ptr(), stream.cuda_stream,
                                counters=True, device=local)
    tr = timed_region(spp, 1)
    elapsed = tr["elapsed"]
    progress(f"timed {args.steps} steps: {elapsed / args.steps * 1e3:.3f} ms/step")
    rccl_ms = tr["rccl_ms"]
    samples = world * args.steps * W * H * spp
    value = samples / elapsed / 1e6
    avg_kernel_s = tr["kernel_s"]
    weak = None
    if world > 1 and cfg["split"]:
        # secondary: every rank renders the whole frame's spp (weak scaling), after the headline region
        wr = timed_region(cfg["spp"], 1 + 2 * (args.warmup + args.steps))
        weak = {"value": round(world * args.steps * W * H * cfg["spp"] / wr["elapsed"] / 1e6, 3),
                "unit": "Msamples/s", "ms_per_step": round(wr["elapsed"] / args.steps * 1e3, 3),
                "spp_per_gpu": cfg["spp"], "render_kernel_ms": round(wr["kernel_s"] * 1e3, 3),
                "scaling": "weak"}
        progress(f"weak: {weak['ms_per_step']} ms/step")
    sequential = None
    if nstreams > 1:
        # the same frames strictly one after another (one stream): each frame's own latency
        sr = timed_region(spp, 1 + 4 * (args.warmup + args.steps), ns=1)
        sequential = {"value": round(samples / sr["elapsed"] / 1e6, 3), "unit": "Msamples/s", "streams": 1,
                      "ms_per_step": round(sr["elapsed"] / args.steps * 1e3, 3),
                      "render_kernel_ms": round(sr["kernel_s"] * 1e3, 3)}
        progress(f"sequential: {sequential['ms_per_step']} ms/step")
        # the roofline's kernel time from launches that do not overlap another frame's
        avg_kernel_s = sr["kernel_s"]
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
                   "parallelism": f"spp-split x{world}, RCCL reduce", "streams": nstreams,
                   "pmc_key": config_key(cfg["scene"], W, H, spp)},
    }
    # samples of 8x8 blocks whose camera rays all miss every object (block_cull_kernel) are applied
    # as the photon {0, 0} without tracing: the records are bit-identical with VR_LAUNCH_NO_CULL
    # (tests/test_gpu_cull.py); every sample is counted in `value`, the traced ones here
    out["traced_msamples_per_s"] = round(world * args.steps * counts["samples"] / elapsed / 1e6, 3)
    if weak:
        out["weak_scaling"] = weak
    if sequential:
        out["sequential"] = sequential
    pmc = None
    if rank == 0 and not args.no_pmc:
        # this rank's shard (at N > 1 too: the PMC child is a one-process run of the same spp)
        child = ["--config", args.config, "--width", str(W), "--height", str(H), "--spp", str(spp),
                 "--scene", cfg["scene"]] + (["--mesh", args.mesh] if args.mesh else []) + \
                (["--host-build"] if args.host_build else [])
        pmc = live_pmc(child)
    out["roofline"] = roofline(counts, W * H, avg_kernel_s, config_key(cfg["scene"], W, H, spp), tr["passes"], pmc)
    if world > 1:
        out["roofline"]["shard"] = f"rank 0's {spp} spp of the {cfg['spp'] if cfg['split'] else spp * world} spp frame"
    out["scene_build"] = build
    # the path's one exchange: {sum X, Y, Z, weight} of every pixel, 32 B, reduced
    # onto rank 0 inside the timed step (RCCL; under torch.distributed.run also at world size 1)
    if args.one_gpu_rehearsal:
        out["rehearsal"] = (f"{world} ranks sharing ONE GPU, gloo reduce of host copies: the N-rank code path, "
                            f"not a multi-GPU measurement")
    out["reduce"] = {"collective": "dist.reduce(SUM, f64) onto rank 0" if distributed else "none (one process)",
                     "bytes_per_step_per_rank": D.reduce_bytes(state) if distributed else 0,
                     "ms_per_step": round(sum(rccl_ms) / len(rccl_ms), 3) if rccl_ms else 0.0}
    out["roofline"]["reduce_kernel_ms"] = round(tr["reduce_ms"], 3)
    out["roofline"]["frustum_culled_sample_fraction"] = round(1.0 - counts["samples"] / (W * H * spp), 4)
    if rank == 0 and world == 1 and not args.no_drop_in:
        progress("drop-in leg")
        out["drop_in"] = drop_in_leg(dscene, W, H, args.drop_in_frames, args.drop_in_threads, local)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        ci = cpu_info()
        threads = args.cpu_threads or ci["usable"]
        progress(f"CPU baseline on {threads} threads")
        out["cpu_baseline"] = cpu_baseline(scene, W, H, args.cpu_seconds, threads)
        out["cpu_baseline"]["host"] = ci
    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        dist.barrier()  # the other ranks wait for rank 0's PMC passes before the group goes away
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)

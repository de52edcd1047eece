"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) for the render kernel into
profiles/<round>/pmc_summary.json and profiles/pmc_traffic.json (read by bench.py).

HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KB units from rocprofv3; FETCH_SIZE doubled
per the gfx950 caveat in MI355X_MICROARCH.md "HBM": it tallies 128-B requests at 64 B).
"""
import collections
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(pass_dir, kernel_substr):
    rows = list(csv.DictReader(open(os.path.join(pass_dir, "run_counter_collection.csv"))))
    per_dispatch = collections.defaultdict(dict)
    for r in rows:
        if kernel_substr in r["Kernel_Name"] and "true" not in r["Kernel_Name"].split("render_kernel<")[-1][:20]:
            per_dispatch[int(r["Dispatch_Id"])].setdefault(r["Counter_Name"], 0.0)
            per_dispatch[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    return per_dispatch


def main():
    pmc = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc")
    out_dir = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "r01")
    args = open(os.path.join(pmc, "args.txt")).read().strip() if os.path.exists(os.path.join(pmc, "args.txt")) else ""
    summary = {"bench_args": args, "kernel": "vr::dev::render_kernel<.., COUNT=false, ..>", "passes": {}}
    for d in sorted(glob.glob(os.path.join(pmc, "*/"))):
        name = os.path.basename(d.rstrip("/"))
        try:
            disp = load(d, "render_kernel")
        except FileNotFoundError:
            continue
        if not disp:
            continue
        last = disp[max(disp)]  # the timed step's dispatch (after the counting launch)
        summary["passes"][name] = last
    f = summary["passes"].get("fetch", {}).get("FETCH_SIZE")
    w = summary["passes"].get("write", {}).get("WRITE_SIZE")
    lib = os.path.join(ROOT, "vanrijn_amd", "lib", "libvanrijn_amd.so")
    sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()
    if f is not None and w is not None:
        summary["hbm_bytes_per_launch"] = 2 * f * 1024 + w * 1024
        summary["fetch_size_kb"] = f
        summary["write_size_kb"] = w
    tcc = summary["passes"].get("tcc", {})
    if tcc.get("TCC_HIT_sum"):
        summary["l2_hit_rate"] = tcc["TCC_HIT_sum"] / (tcc["TCC_HIT_sum"] + tcc["TCC_MISS_sum"])
    summary["lib_sha256"] = sha
    os.makedirs(out_dir, exist_ok=True)
    json.dump(summary, open(os.path.join(out_dir, "pmc_summary.json"), "w"), indent=1)
    if "hbm_bytes_per_launch" in summary:
        cfg = {"width": 1024, "height": 1024, "spp": 256, "scene": "main"}
        toks = args.split()
        for k in cfg:
            if f"--{k}" in toks:
                cfg[k] = toks[toks.index(f"--{k}") + 1]
        config = f"--width {cfg['width']} --height {cfg['height']} --spp {cfg['spp']} --scene {cfg['scene']}"
        json.dump({"lib_sha256": sha, "config": config, "hbm_bytes_per_launch": summary["hbm_bytes_per_launch"],
                   "source": os.path.relpath(os.path.join(out_dir, "pmc_summary.json"), ROOT)},
                  open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()

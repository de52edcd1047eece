"""Fold rocprofv3 --pmc passes (tools/pmc.sh) of the render kernel into a PMC record.

    python tools/pmc_summary.py gpurun_out/pmc/<name> profiles/<round>/pmc_<name>.json

Writes the full summary to the second path and adds / replaces the record of this library build
and bench config in profiles/pmc_records.json, which bench.py reads for its roofline:
  per_launch  every counter of the timed render_kernel dispatch (COUNT=false), summed over the
              rows rocprofv3 writes for it;
  kernel_ns   that dispatch's duration in the tcc pass (GRBM_GUI_ACTIVE / 8 / kernel_ns = clock);
HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KB units; FETCH_SIZE doubled per the gfx950
caveat in MI355X_MICROARCH.md: it tallies 128-B requests at 64 B).
"""
import collections
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def is_timed_render(name):
    # render_kernel<STACK, COUNT, RECORD, ...>: the timed launches have COUNT = false
    if "render_kernel<" not in name:
        return False
    targs = name.split("render_kernel<")[1].split(">")[0].split(",")
    return targs[1].strip() == "false" and targs[2].strip() == "false"


def load(pass_dir):
    rows = list(csv.DictReader(open(os.path.join(pass_dir, "run_counter_collection.csv"))))
    per = collections.defaultdict(dict)
    for r in rows:
        if is_timed_render(r["Kernel_Name"]):
            d = per[int(r["Dispatch_Id"])]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    durations = {}
    trace = os.path.join(pass_dir, "run_kernel_trace.csv")
    if os.path.exists(trace):
        for r in csv.DictReader(open(trace)):
            if is_timed_render(r["Kernel_Name"]):
                durations[int(r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return per, durations


def bench_key(pmc_dir):
    for f in sorted(glob.glob(os.path.join(pmc_dir, "*.out"))):
        for line in open(f):
            line = line.strip()
            if line.startswith("{"):
                return json.loads(line)["config"]["pmc_key"]
    raise SystemExit("no bench JSON line in the pass outputs")


def main():
    pmc_dir, out_path = sys.argv[1], sys.argv[2]
    per_launch, kernel_ns = {}, {}
    for d in sorted(glob.glob(os.path.join(pmc_dir, "*/"))):
        name = os.path.basename(d.rstrip("/"))
        if not os.path.exists(os.path.join(d, "run_counter_collection.csv")):
            continue
        disp, dur = load(d)
        if not disp:
            continue
        last = max(disp)  # the timed step's dispatch (after the counting launch)
        per_launch.update(disp[last])
        if last in dur:
            kernel_ns[name] = dur[last]
    sha_file = os.path.join(pmc_dir, "lib.sha256")  # written on the box by tools/pmc.sh
    if os.path.exists(sha_file):
        sha = open(sha_file).read().strip()
    else:
        lib = os.path.join(ROOT, "vanrijn_amd", "lib", "libvanrijn_amd.so")
        sha = sys.argv[3] if len(sys.argv) > 3 else hashlib.sha256(open(lib, "rb").read()).hexdigest()
    key = bench_key(pmc_dir)
    rec = {"lib_sha256": sha, "config": key, "per_launch": per_launch,
           "kernel_ns": kernel_ns.get("tcc") or max(kernel_ns.values()),
           "kernel_ns_per_pass": kernel_ns, "bench_args": open(os.path.join(pmc_dir, "args.txt")).read().strip(),
           "source": os.path.relpath(out_path, ROOT)}
    rec["hbm_bytes_per_launch"] = 2 * per_launch["FETCH_SIZE"] * 1024 + per_launch["WRITE_SIZE"] * 1024
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    json.dump(rec, open(out_path, "w"), indent=1)
    recs_path = os.path.join(ROOT, "profiles", "pmc_records.json")
    try:
        recs = json.load(open(recs_path))
    except (OSError, ValueError):
        recs = {}
    recs[key] = rec
    json.dump(recs, open(recs_path, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: rec[k] for k in ("config", "kernel_ns", "hbm_bytes_per_launch", "lib_sha256")}))


if __name__ == "__main__":
    main()

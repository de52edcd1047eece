#!/bin/bash
# A/B of two library builds (abx/lib$A.so, abx/lib$B.so): the parity tests on B, then interleaved
# per-process timings and record digests (tools/lib_ab.py) on C3, C5-sized, C2 and C1
#   A=base B=tri128 OUT=gpurun_out/x bash tools/r06_libab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06ab}
A=${A:-base}
B=${B:?name of the B build}
mkdir -p "$O"
export TMPDIR=/tmp
VR_LIBRARY=abx/lib$B.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/parity_$B.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$O/parity_$B.log"; exit 1; }
tail -1 "$O/parity_$B.log"
for sc in "main 1024 256 3" "c5 2048 16 3" "main 512 64 5" "bench 256 16 9"; do
  for r in 1 2; do
    for lib in $A $B; do
      VR_LIBRARY=abx/lib$lib.so timeout -k 10 300 python tools/lib_ab.py $sc >> "$O/ab.jsonl" 2>> "$O/err" || { echo rc=$?; tail "$O/err"; exit 1; }
    done
  done
done
python3 - "$O/ab.jsonl" <<'PY'
import json, sys, collections, statistics
rows = [json.loads(l) for l in open(sys.argv[1])]
g = collections.defaultdict(list)
dig = collections.defaultdict(set)
for r in rows:
    k = (r["scene"], r["size"], r["spp"])
    g[(k, r["lib"])].append(r["median_ms"])
    dig[k].add(r["digest"])
for (k, lib), v in sorted(g.items()):
    print(k, lib, round(statistics.mean(v), 3), "digests equal" if len(dig[k]) == 1 else "DIGESTS DIFFER")
PY

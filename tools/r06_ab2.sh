#!/bin/bash
# a longer interleaved A/B of two builds on C3 (1024^2 @256) and C5's frame (4096^2 @8):
#   A=base B=trk OUT=gpurun_out/x bash tools/r06_ab2.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06ab2}
A=${A:-base}
B=${B:?name of the B build}
mkdir -p "$O"
export TMPDIR=/tmp
for sc in "main 1024 256 3" "c5 4096 8 3"; do
  for r in 1 2 3 4; do
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
    print(k, lib, round(statistics.mean(v), 3), [round(x, 2) for x in v], "digests equal" if len(dig[k]) == 1 else "DIGESTS DIFFER")
PY

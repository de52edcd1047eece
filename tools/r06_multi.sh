#!/bin/bash
# several builds against abx/libbase.so on one configuration, interleaved per process:
#   LIBS="base x y" SC="main 1024 256 3" ROUNDS=3 OUT=gpurun_out/x bash tools/r06_multi.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06multi}
mkdir -p "$O"
export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-3}); do
  for lib in ${LIBS:?}; do
    VR_LIBRARY=abx/lib$lib.so timeout -k 10 300 python tools/lib_ab.py ${SC:-main 1024 256 3} >> "$O/ab.jsonl" 2>> "$O/err" || { echo rc=$?; tail "$O/err"; exit 1; }
  done
done
python3 - "$O/ab.jsonl" <<'PY'
import json, sys, collections, statistics
rows = [json.loads(l) for l in open(sys.argv[1])]
g = collections.defaultdict(list)
red = collections.defaultdict(list)
dig = collections.defaultdict(set)
for r in rows:
    k = (r["scene"], r["size"], r["spp"])
    g[(k, r["lib"])].append(r["median_ms"])
    red[(k, r["lib"])].append(r.get("reduce_ms", 0.0))
    dig[k].add(r["digest"])
for (k, lib), v in sorted(g.items()):
    print(k, lib, round(statistics.mean(v), 3), [round(x, 2) for x in v], "reduce", round(statistics.mean(red[(k, lib)]), 3), "digests equal" if len(dig[k]) == 1 else "DIGESTS DIFFER")
PY

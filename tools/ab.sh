#!/bin/bash
# A/B library builds on the GPU box: alternating processes, main 256 spp + bench 32 spp per library.
#   ROUNDS=3 bash tools/ab.sh path/to/libA.so path/to/libB.so [more libraries ...]
# SCENES: "scene:spp[:size] ..." (default "main:256 bench:32", size 1024)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=${ROUNDS:-3}
: > gpurun_out/ab_libs.jsonl
SCENES=${SCENES:-"main:256 bench:32"}
[ "${BENCH_SCENE:-1}" = 1 ] || SCENES="main:256"
for r in $(seq 1 "$R"); do
  for L in "$@"; do
    for sc in $SCENES; do
      IFS=: read -r SC SPP SZ <<< "$sc"
      VR_LIBRARY="$L" timeout -k 10 300 python tools/variants.py --scene $SC --spp $SPP --size ${SZ:-1024} --reps 2 --variants 0 \
          --thresholds 52 2>> gpurun_out/variants.err | sed "s|^|$(basename "$L") |" >> gpurun_out/ab_libs.jsonl
      rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }
    done
  done
  echo "round $r done"
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for line in open("gpurun_out/ab_libs.jsonl"):
    name, js = line.split(" ", 1)
    r = json.loads(js)
    d[(r["scene"], name)].append((r["median_ms"], r.get("reduce_ms", 0.0)))
for k, v in sorted(d.items()):
    ms = sorted(x[0] for x in v)
    red = sorted(x[1] for x in v)
    print(k, "median of medians %.3f ms (reduce %.3f ms)" % (ms[len(ms) // 2], red[len(red) // 2]),
          ["%.2f" % x[0] for x in v])
PY

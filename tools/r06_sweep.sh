#!/bin/bash
# threshold sweeps on the two-step kernel (tuning build abx/libtune2.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06sw}
mkdir -p "$O"
export TMPDIR=/tmp
export VR_LIBRARY=abx/libtune2.so
run() { timeout -k 10 400 python tools/variants.py "$@" >> "$O/sw.jsonl" 2>> "$O/err" || { echo rc=$?; tail "$O/err"; exit 1; }; }
run --scene main --spp 256 --size 1024 --reps 3 --variants 0 --thresholds 44,48,52,56,60
run --scene main --spp 256 --size 1024 --reps 3 --variants 0 --thresholds 52 --env VR_LEAF_THRESHOLD=40,48,56,64
run --scene main --spp 256 --size 1024 --reps 3 --variants 0 --thresholds 52 --env VR_LEAF_STALL=2,3,4,6
run --scene c5 --spp 16 --size 2048 --reps 3 --variants 0 --thresholds 44,48,52,56,60
python3 - <<'PY'
import json
for l in open("gpurun_out/r06sw/sw.jsonl"):
    d=json.loads(l); print({k:v for k,v in d.items() if k in ("scene","threshold","VR_LEAF_THRESHOLD","VR_LEAF_STALL","median_ms","bitwise_equal_to_first")})
PY

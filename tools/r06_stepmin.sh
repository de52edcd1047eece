#!/bin/bash
# extra node steps gated on the lanes at a node (tuning builds abx/libtune2.so, abx/libtune3.so: VR_STEP_MIN)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06sm}
mkdir -p "$O"
export TMPDIR=/tmp
for L in tune2 tune3; do
  for sc in "main --spp 256 --size 1024" "c5 --spp 16 --size 2048"; do
    set -- $sc
    VR_LIBRARY=abx/lib$L.so timeout -k 10 300 python tools/variants.py --scene $1 $2 $3 $4 $5 --reps 3 --variants 0 --thresholds 52 --env VR_STEP_MIN=1,8,16,32 | sed "s/^/$L /" >> "$O/sm.jsonl" 2>> "$O/err" || { echo rc=$?; tail "$O/err"; exit 1; }
  done
done
cut -c1-150 "$O/sm.jsonl"

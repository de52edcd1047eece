#!/bin/bash
# node steps per phase-B iteration: compile-time 2 (abx/libsteps2.so) against the runtime count
# (abx/librt.so, VR_NODE_STEPS=1/2/3 in one process) on C3 and C5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06st}
mkdir -p "$O"
export TMPDIR=/tmp
for sc in "main --spp 256 --size 1024" "c5 --spp 16 --size 2048" "main --spp 64 --size 512"; do
  set -- $sc
  VR_LIBRARY=abx/librt.so timeout -k 10 300 python tools/variants.py --scene $1 $2 $3 $4 $5 --reps 3 --variants 0 --thresholds 52 --env VR_NODE_STEPS=1,2,3 >> "$O/rt.jsonl" 2>> "$O/err" || { echo rc=$?; tail "$O/err"; exit 1; }
  VR_LIBRARY=abx/libsteps2.so timeout -k 10 300 python tools/variants.py --scene $1 $2 $3 $4 $5 --reps 3 --variants 0 --thresholds 52 >> "$O/ct2.jsonl" 2>> "$O/err" || { echo rc=$?; tail "$O/err"; exit 1; }
done
cat "$O/rt.jsonl" "$O/ct2.jsonl" | cut -c1-200

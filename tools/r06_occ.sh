#!/bin/bash
# Occupancy A/B of the production render kernel (tuning build): 16-bit LDS stack entries at 3 and 4 waves
# per SIMD (variants 6 / 5; 4 workgroups per CU for variant 5) against the default (variant 0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06o}
mkdir -p "$O"
export TMPDIR=/tmp
export VR_LIBRARY=abx/libtune.so
for spp in 256 64; do
  timeout -k 10 400 python tools/variants.py --spp $spp --reps 3 --variants 0,6 --thresholds 52 > "$O/occ3_$spp.jsonl" 2> "$O/occ.err" || { echo "occ3 rc=$?"; tail "$O/occ.err"; exit 1; }
  VR_GRID_PER_CU=4 timeout -k 10 400 python tools/variants.py --spp $spp --reps 3 --variants 5 --thresholds 52 > "$O/occ4_$spp.jsonl" 2>> "$O/occ.err" || { echo "occ4 rc=$?"; tail "$O/occ.err"; exit 1; }
  cat "$O/occ3_$spp.jsonl" "$O/occ4_$spp.jsonl"
done

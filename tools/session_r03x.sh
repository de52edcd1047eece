#!/bin/bash
# Round-3 GPU session X: phase-threshold sweeps on the DP-collapse build (one process per sweep,
# main scene 1024^2 @256, records bitwise-checked across settings), and the ordered reduce with 2
# samples per colour batch (VR_REDUCE_BATCH=2: occupancy 5 instead of 4) against the default (4).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03x}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
sw() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python tools/variants.py --scene main --spp 256 --reps 3 --variants 0 "$@" > $O/sweep_$n.jsonl 2>> $O/sweep.err
  ok $? "sweep $n"
  python3 -c "
import json,sys
for l in open('$O/sweep_$n.jsonl'):
    r=json.loads(l); k={a:b for a,b in r.items() if a not in ('variant','scene','min_ms','reduce_ms','msamples_s')}
    print('$n', k)"
}
sw shade --thresholds 44,48,52,56,60
sw leaf --thresholds 52 --env VR_LEAF_THRESHOLD=40,44,48,52,56
sw stall --thresholds 52 --env VR_LEAF_STALL=2,3,4,5
sw shademin --thresholds 52 --env VR_SHADE_MIN=8,12,16,20,24
sw missmin --thresholds 52 --env VR_MISS_MIN=4,8,12,16
SCENES="main:256" ROUNDS=3 timeout -k 10 600 bash tools/ab.sh abx/libcur.so abx/libkb2.so > $O/ab_kb2.txt 2>&1; ok $? ab; tail -3 $O/ab_kb2.txt

#!/bin/bash
# One-dimensional sweeps of the render kernel's tuning knobs around the defaults, main.rs scene
# 1024^2 @256 (tuning build: bash tools/build_variant.sh tune -DVR_TUNING_VARIANTS; abx/libtune.so).
#   bash tools/sweep_main.sh [scene spp size]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SC=${1:-main}; SPP=${2:-256}; SZ=${3:-1024}
O=gpurun_out/sweep; mkdir -p $O
export VR_LIBRARY=abx/libtune.so
run() { timeout -k 10 240 python tools/variants.py --scene $SC --spp $SPP --size $SZ --reps 3 --variants 0 "$@" >> $O/${SC}.jsonl 2>> $O/err.log; }
: > $O/${SC}.jsonl
run --thresholds 40,44,48,52,56,60 || exit 1
run --thresholds 52 --env VR_LEAF_THRESHOLD=32,40,48,56,64 || exit 1
run --thresholds 52 --env VR_LEAF_STALL=2,3,4,6 || exit 1
run --thresholds 52 --env VR_MISS_MIN=0,4,8,16 || exit 1
run --thresholds 52 --env VR_SHADE_MIN=8,12,16,24,32 || exit 1
run --thresholds 52 --env VR_PHASE_A_REPS=1,2,3 || exit 1
run --thresholds 52 --env VR_GRAB=256,384,512,768 || exit 1
cat $O/${SC}.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); k={x:d[x] for x in d if x.startswith('VR_')}
    print(d['threshold'], k, round(d['median_ms'],3), d['bitwise_equal_to_first'])"

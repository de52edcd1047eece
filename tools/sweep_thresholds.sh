#!/bin/bash
# Threshold sweeps of the render kernel (tools/variants.py, in-process) on one scene:
#   SCENE=main SPP=64 bash tools/sweep_thresholds.sh   (results: gpurun_out/sw_*_$SCENE.txt)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
sc=${SCENE:-main}; spp=${SPP:-64}
timeout -k 10 240 python tools/variants.py --scene $sc --spp $spp --reps 3 --variants 0 --thresholds 52 --env VR_LEAF_THRESHOLD=40,48,56 --env VR_LEAF_STALL=2,3,4 > gpurun_out/sw_leaf_$sc.txt 2>/dev/null
timeout -k 10 240 python tools/variants.py --scene $sc --spp $spp --reps 3 --variants 0 --thresholds 44,48,52,56 --env VR_SHADE_MIN=8,16,24 > gpurun_out/sw_shade_$sc.txt 2>/dev/null
timeout -k 10 240 python tools/variants.py --scene $sc --spp $spp --reps 3 --variants 0 --thresholds 52 --env VR_PHASE_A_REPS=1,2,3 --env VR_MISS_MIN=4,8,16 > gpurun_out/sw_misc_$sc.txt 2>/dev/null

#!/bin/bash
# Round-3 GPU session M: wave-uniform refill decode (a slice's (chunk, live block) pairs stepped in
# scalar registers, live blocks packed as (row, column)): the -m gpu suite on this build, the A/B
# against the previous default build, and the small frames (C1, C2) of both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03m}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; ok $rc gpu-tests
cp vanrijn_amd/lib/libvanrijn_amd.so abx/librefill.so
SCENES="main:256 bench:32 c5:16" ROUNDS=3 timeout -k 10 900 bash tools/ab.sh abx/libhot0.so abx/librefill.so \
    > $O/ab_refill.txt 2>&1; ok $? ab; tail -6 $O/ab_refill.txt
cp gpurun_out/ab_libs.jsonl $O/ab_refill.jsonl
for L in abx/libhot0.so abx/librefill.so abx/libhot0.so abx/librefill.so; do
  for sc in bench:256:16 main:512:64 main:1024:1; do
    IFS=: read -r scene size spp <<< "$sc"
    VR_LIBRARY=$L timeout -k 10 300 python tools/variants.py --scene $scene --size $size --spp $spp --reps 7 \
        --variants 0 --thresholds 52 2>> $O/variants.err | sed "s|^|$(basename $L) |" >> $O/small_frames.jsonl
    ok $? "small $sc"
  done
done
cut -c 1-150 $O/small_frames.jsonl

#!/bin/bash
# Round-3 GPU session I: the cooperative tail moved out of the node step (abx/libcoop.so): parity of
# the tail-heavy tests, then the A/B against the build without it and the small frames.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03i}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
VR_LIBRARY=abx/libcoop.so timeout -k 10 400 python -u -m pytest tests/test_gpu_build.py tests/test_gpu_parity.py \
    tests/test_gpu_fullframe.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/coop_tests.log 2>&1
rc=$?; tail -3 $O/coop_tests.log; ok $rc coop-tests
SCENES="main:256 bench:32 c5:16" ROUNDS=3 timeout -k 10 900 bash tools/ab.sh abx/libbase.so abx/libcoop.so \
    > $O/ab_coop.txt 2>&1; ok $? ab; tail -7 $O/ab_coop.txt
for L in abx/libbase.so abx/libcoop.so; do
  for sc in bench:256:16 main:1024:1; do
    IFS=: read -r scene size spp <<< "$sc"
    VR_LIBRARY=$L timeout -k 10 300 python tools/variants.py --scene $scene --size $size --spp $spp --reps 7 \
        --variants 0 --thresholds 52 | sed "s|^|$(basename $L) |" >> $O/small_frames.jsonl 2>> $O/variants.err
    ok $? "small $sc"
  done
done
cut -c 1-160 $O/small_frames.jsonl

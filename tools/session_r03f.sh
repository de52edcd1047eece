#!/bin/bash
# Round-3 GPU session F: the device SAH build (tests, then device vs host tree on main and C5),
# the per-sphere near-unit reciprocal A/B, and the full -m gpu suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03f}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_build.py -x -v -s --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/gpu_build_tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|build:" $O/gpu_build_tests.log | tail -25; ok $rc build-tests
for c in "main 1024 64" "c5 1024 16" "c5 4096 4"; do
  timeout -k 10 300 python tools/sah_ab.py $c 3 >> $O/sah_ab.jsonl 2>> $O/sah_ab.err; ok $? "sah ab $c"
done
cut -c 1-600 $O/sah_ab.jsonl
SCENES="main:256 bench:32 c5:16" ROUNDS=3 timeout -k 10 900 bash tools/ab.sh abx/libbase.so abx/libnear1.so \
    > $O/ab_near1.txt 2>&1; ok $? ab; tail -7 $O/ab_near1.txt
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; ok $rc gpu-tests
for c in "bench 256 16" "main 1024 1"; do
  timeout -k 10 300 python tools/longpath.py $c >> $O/longpath.jsonl 2>> $O/longpath.err; ok $? "longpath $c"
done
cat $O/longpath.jsonl
for sc in bench:256:16 main:1024:1 main:1024:64; do
  IFS=: read -r scene size spp <<< "$sc"
  timeout -k 10 400 python tools/variants.py --scene $scene --size $size --spp $spp --reps 3 --variants 0 \
      --thresholds 52 --env VR_LEAF_FEW=0,4,8,16,64 >> $O/sweep_leaf_few_tail.jsonl 2>> $O/variants.err; ok $? "sweep $sc"
done
cut -c 1-160 $O/sweep_leaf_few_tail.jsonl

#!/bin/bash
# Round-3 GPU session K: LDS copy of the tree's top (VR_HOT_MAX): parity of the hot build, the A/B
# against HEAD and the no-LDS build of the same source.  (A PC-sampling step that followed was
# refused by the pool's profiler policy; it is not run.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03k}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
VR_LIBRARY=abx/libhot32.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullframe.py \
    tests/test_gpu_build.py tests/test_gpu_cull.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > $O/hot_tests.log 2>&1
rc=$?; tail -3 $O/hot_tests.log; ok $rc hot-tests
SCENES="main:256 bench:32 c5:16" ROUNDS=3 timeout -k 10 1000 bash tools/ab.sh abx/libhead.so abx/libhot0.so \
    abx/libhot32.so abx/libhot16.so > $O/ab_hot.txt 2>&1; ok $? ab; tail -12 $O/ab_hot.txt
cp gpurun_out/ab_libs.jsonl $O/ab_hot.jsonl

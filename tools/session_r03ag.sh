#!/bin/bash
# Round-3 GPU session AG: the ordered reduce with the next batch's loads issued before this batch's
# colours (VR_REDUCE_PREFETCH) against the same source without it; the cull/reduce parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03ag}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_cull.py tests/test_gpu_fullframe.py tests/test_gpu_parity.py -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1; rc=$?; tail -2 $O/gpu_tests.log; ok $rc tests
SCENES="main:256 main:64" ROUNDS=3 timeout -k 10 900 bash tools/ab.sh abx/libnopf.so abx/libpf.so > $O/ab_pf.txt 2>&1; ok $? ab
tail -3 $O/ab_pf.txt

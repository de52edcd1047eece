#!/bin/bash
# Round-3 GPU session AJ: the hardened frustum-cull test on the closing build (must pass) and on the
# b38f898 build whose cut tiles read stale staging (must fail: the test's sensitivity).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03aj}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_cull.py -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > $O/cull_closing.log 2>&1; rc1=$?; tail -2 $O/cull_closing.log; echo "closing build rc=$rc1"
[ $rc1 -eq 0 ] || exit $rc1
VR_LIBRARY=abx/lib_b38f898.so timeout -k 10 300 python -u -m pytest tests/test_gpu_cull.py -v --timeout 200 \
    --timeout-method thread -p no:cacheprovider > $O/cull_b38f898.log 2>&1; rc2=$?; tail -2 $O/cull_b38f898.log
echo "b38f898 build rc=$rc2 (expected: failures)"
exit 0

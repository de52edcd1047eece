#!/bin/bash
# A/B the working-tree library against abx/lib<BASE>.so, then the GPU tests on the working tree.
#   BASE=base ROUNDS=3 TESTS=1 bash tools/session_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 bash tools/ab.sh abx/lib${BASE:-base}.so vanrijn_amd/lib/libvanrijn_amd.so ${ROUNDS:-3} > gpurun_out/ab_summary.txt 2>&1
rc=$?; cat gpurun_out/ab_summary.txt; [ $rc -eq 0 ] || exit $rc
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
      > gpurun_out/ab_gpu_tests.log 2>&1
  rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/ab_gpu_tests.log; exit $rc
fi

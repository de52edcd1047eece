#!/bin/bash
# A/B the libraries under abx/ (tools/variant_libs.sh), then optionally the GPU tests on the working tree.
#   LIBS="base node1" ROUNDS=3 TESTS=1 bash tools/session_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
paths=""
for n in ${LIBS:-base}; do paths="$paths abx/lib$n.so"; done
timeout -k 10 1000 bash tools/ab.sh $paths > gpurun_out/ab_summary.txt 2>&1
rc=$?; cat gpurun_out/ab_summary.txt; [ $rc -eq 0 ] || exit $rc
if [ "${TESTS:-0}" = "1" ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
      > gpurun_out/ab_gpu_tests.log 2>&1
  rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/ab_gpu_tests.log; exit $rc
fi

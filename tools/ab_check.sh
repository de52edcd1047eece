#!/bin/bash
# GPU tests of the working tree, then an A/B of two libraries (tools/ab.sh) -- one gpurun call:
#   SCENES="bench:16:256" bash tools/ab_check.sh abx/libA.so abx/libB.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/abc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
ROUNDS=${ROUNDS:-3} bash tools/ab.sh "$@"

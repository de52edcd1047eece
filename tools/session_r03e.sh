#!/bin/bash
# Round-3 GPU session E: A/B of the sphere hoist (a, 1/(2a) once per ray, near-unit reciprocal) and
# the empty leaf-append skip, alone and together, on the main, bench and C5 scenes; then parity.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03e}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
SCENES="main:256 bench:32 c5:16" ROUNDS=3 timeout -k 10 1200 bash tools/ab.sh abx/libbase.so abx/libhoist.so \
    abx/libskip.so vanrijn_amd/lib/libvanrijn_amd.so > $O/ab_hoist_skip.txt 2>&1; ok $? ab; tail -13 $O/ab_hoist_skip.txt
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; ok $rc gpu-tests

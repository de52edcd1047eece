#!/bin/bash
# Round-3 GPU session O: rotated triangle copies (the leaf round reads its ray's axis order, no
# per-lane component selects), slab32_flags on one difference, mbcnt lane prefixes: the -m gpu
# suite on this build, then the A/B: HEAD (base3), slab + mbcnt (mid), all three (rot).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03o}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; ok $rc gpu-tests
SCENES="main:256 bench:32 c5:16" ROUNDS=3 timeout -k 10 1100 bash tools/ab.sh abx/libbase3.so abx/libmid.so \
    abx/librot.so > $O/ab_rot.txt 2>&1; ok $? ab; tail -9 $O/ab_rot.txt
cp gpurun_out/ab_libs.jsonl $O/ab_rot.jsonl

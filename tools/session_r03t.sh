#!/bin/bash
# Round-3 GPU session T: the leaf round's vertex components loaded in the owner ray's axis order
# (VR_ROT_LOAD, vr_device.h triangle_distance_rot): the -m gpu suite on this build, then the A/B
# against the same source with VR_ROT_LOAD=0 (base4).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03t}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; ok $rc gpu-tests
SCENES="main:256 bench:32 c5:16" ROUNDS=3 timeout -k 10 1100 bash tools/ab.sh abx/libbase4.so abx/librotld.so \
    > $O/ab_rotld.txt 2>&1; ok $? ab; tail -9 $O/ab_rotld.txt
cp gpurun_out/ab_libs.jsonl $O/ab_rotld.jsonl

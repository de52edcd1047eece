#!/bin/bash
# Round-3 GPU session P: votes as compares into lane masks (llvm.amdgcn.icmp / fcmp instead of
# __ballot of a bool, which is lowered to v_cndmask + v_cmp): the -m gpu suite on this build, the
# A/B against the committed build (mid2) and HEAD before the session's kernel changes (base3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03p}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; ok $rc gpu-tests
SCENES="main:256 bench:32 c5:16" ROUNDS=3 timeout -k 10 1100 bash tools/ab.sh abx/libbase3.so abx/libmid2.so \
    abx/libvote.so > $O/ab_vote.txt 2>&1; ok $? ab; tail -9 $O/ab_vote.txt
cp gpurun_out/ab_libs.jsonl $O/ab_vote.jsonl

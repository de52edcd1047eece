#!/bin/bash
# Round-3 GPU session W: the stack-budgeted DP collapse (a node takes the DP expansion where its
# subtree's stack bound keeps the greedy tree's LDS stack class: C5's mesh now DP-collapsed too):
# the -m gpu suite, then the A/B against the greedy collapse on C5 and main.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03w}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; ok $rc gpu-tests
SCENES="c5:16 main:256" ROUNDS=3 timeout -k 10 1000 bash tools/ab.sh abx/libgreedy.so abx/libwidedp2.so \
    > $O/ab_widedp2.txt 2>&1; ok $? ab; tail -5 $O/ab_widedp2.txt
cp gpurun_out/ab_libs.jsonl $O/ab_widedp2.jsonl

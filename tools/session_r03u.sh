#!/bin/bash
# Round-3 GPU session U: SAH-optimal DP collapse of the 4-wide tree (VR_WIDE_DP, vr_host.cpp
# WideBuilder): the -m gpu suite on this build, node visits of both collapses (counting variant),
# the A/B against the greedy collapse (libgreedy).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03u}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; ok $rc gpu-tests
for dp in 1 0; do
  VR_WIDE_STATS=1 VR_WIDE_DP=$dp timeout -k 10 300 python tools/cycles.py 64 main > $O/cycles_main_dp$dp.json 2>> $O/cycles.err
  ok $? cycles-dp$dp
done
grep "vr wide tree" $O/cycles.err
python3 -c "
import json
for dp in (1, 0):
    d = json.load(open('$O/cycles_main_dp%d.json' % dp)); c = d['counters']
    print('dp', dp, 'kernel_ms', round(d['kernel_ms'], 3), 'node_visits', c['node_visits'], 'box_tests', c['box_tests'], 'tri_tests', c['triangle_tests'])
"
SCENES="main:256 bench:32" ROUNDS=3 timeout -k 10 900 bash tools/ab.sh abx/libgreedy.so abx/libwidedp.so \
    > $O/ab_widedp.txt 2>&1; ok $? ab; tail -5 $O/ab_widedp.txt
cp gpurun_out/ab_libs.jsonl $O/ab_widedp.jsonl

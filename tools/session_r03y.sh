#!/bin/bash
# Round-3 GPU session Y: the stack-budgeted DP collapse on C5's 1.05 M-triangle mesh (A/B against the
# greedy collapse), and the C4 / C5 bench lines on one GPU (BASELINE configs[3] / [4]).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03y}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
SCENES="c5:16" ROUNDS=3 timeout -k 10 900 bash tools/ab.sh abx/libgreedy.so abx/libcur.so > $O/ab_c5_dp.txt 2>&1; ok $? ab
tail -2 $O/ab_c5_dp.txt
cp gpurun_out/ab_libs.jsonl $O/ab_c5_dp.jsonl
for c in c5 c4; do
  timeout -k 10 600 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-drop-in --no-pmc \
      > $O/bench_$c.json 2> $O/bench_$c.err; ok $? bench-$c
  cut -c 1-330 $O/bench_$c.json
done

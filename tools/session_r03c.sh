#!/bin/bash
# Round-3 GPU session C: opcode costs (+ v_mul_f32, cndmask forms), the default bench line with
# live PMC, section cycles of the current build, and the small-frame tail diagnostics (C1, 1 spp).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03c}
mkdir -p $O
sha256sum vanrijn_amd/lib/libvanrijn_amd.so > $O/lib.sha256
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }

timeout -k 10 240 tools/opcost 2048 > $O/opcost.json 2> $O/opcost.err; ok $? opcost
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
cut -c 1-300 $O/bench_default.json; tail -3 $O/bench_default.err; ok $rc bench
timeout -k 10 300 python tools/cycles.py 64 main > $O/cycles_main_64spp.json 2> $O/cycles.err; ok $? cycles
for cfg in "bench 256 16" "main 1024 1" "main 512 64"; do
  timeout -k 10 300 python tools/tail.py $cfg >> $O/tail.jsonl 2>> $O/tail.err; ok $? "tail $cfg"
done
cut -c 1-400 $O/tail.jsonl

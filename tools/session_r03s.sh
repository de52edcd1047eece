#!/bin/bash
# Round-3 session s: GPU tests, the default bench (deferred timing), section cycles with the node-step
# histogram (main 64 spp), the long-path breakdown of the bench scene (C1) and the main scene.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
ok() { [ "$1" -eq 0 ] || { echo "$2 failed rc=$1"; exit "$1"; }; echo "$2 ok"; }
sha256sum vanrijn_amd/lib/libvanrijn_amd.so > $O/lib.sha256
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1; ok $? tests
tail -2 $O/gpu_tests.log
timeout -k 10 600 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err; ok $? bench
cut -c 1-300 $O/bench_c3.json
timeout -k 10 300 python tools/cycles.py 64 main > $O/cycles_main_64spp.json 2> $O/cycles.err; ok $? cycles
timeout -k 10 300 python tools/longpath.py bench 256 16 > $O/longpath.jsonl 2>> $O/longpath.err; ok $? longpath
cat $O/longpath.jsonl

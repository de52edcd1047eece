#!/bin/bash
# Round-3 GPU session L: 8-B staged photons (intensity only; the reduce re-draws the wavelength,
# a mask bit marks the recursion limit's lambda 0): the -m gpu suite on this build, the A/B against
# the 16-B staging build, and the default bench line (its live PMC passes give WRITE_SIZE).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03l}
mkdir -p $O
sha256sum vanrijn_amd/lib/libvanrijn_amd.so > $O/lib.sha256
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; ok $rc gpu-tests
SCENES="main:256 bench:32 c5:16" ROUNDS=3 timeout -k 10 900 bash tools/ab.sh abx/libhot0.so \
    vanrijn_amd/lib/libvanrijn_amd.so > $O/ab_stage8.txt 2>&1; ok $? ab; tail -6 $O/ab_stage8.txt
cp gpurun_out/ab_libs.jsonl $O/ab_stage8.jsonl
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
cut -c 1-300 $O/bench_default.json; tail -3 $O/bench_default.err; ok $rc bench

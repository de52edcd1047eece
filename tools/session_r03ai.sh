#!/bin/bash
# Round-3 GPU session AI: the kernel sources restored to 31bf95a (two-owner coop and reduce prefetch
# removed): the cut-tile cull check three times, the -m gpu suite, smoke and the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03ai}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
sha256sum vanrijn_amd/lib/libvanrijn_amd.so > $O/lib.sha256
for i in 1 2 3; do timeout -k 10 120 python tools/debug_cull_pf.py 2>&1 | grep "differing" ; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1; rc=$?; tail -2 $O/gpu_tests.log; ok $rc gpu-tests
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; ok $rc smoke
timeout -k 10 600 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err; ok $? bench
cut -c 1-250 $O/bench_c3.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-drop-in --no-pmc > $O/prof_bench.json 2> $O/prof.err
ok $? rocprof

#!/bin/bash
# Round-3 GPU session B: opcode costs (per-SIMD span), the -m gpu suite (full-frame and NaN
# parity, two-process shards), the default bench line with its live PMC passes, the torchrun
# world-1 rehearsal of the 32-B reduce, and a kernel-trace summary of the default command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03b}
mkdir -p $O
sha256sum vanrijn_amd/lib/libvanrijn_amd.so > $O/lib.sha256
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }

if [ "${OPCOST:-1}" = 1 ]; then
  timeout -k 10 180 tools/opcost 2048 > $O/opcost.json 2> $O/opcost.err; ok $? opcost
fi
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
    --durations=15 > $O/gpu_tests.log 2>&1; rc=$?; tail -22 $O/gpu_tests.log; ok $rc gpu-tests
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
cut -c 1-600 $O/bench_default.json; tail -3 $O/bench_default.err; ok $rc bench
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --steps 2 --warmup 1 --no-cpu-baseline --no-drop-in --no-pmc \
    > $O/bench_torchrun1.json 2> $O/bench_torchrun1.err; rc=$?; tail -2 $O/bench_torchrun1.err; ok $rc torchrun-world1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_default -o run -- \
    python bench.py --no-pmc > $O/prof_default_bench.json 2> $O/prof_default.err; ok $? rocprof-default

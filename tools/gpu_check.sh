#!/bin/bash
# One GPU session: parity tests, a bench line, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash / abort / timeout ends the session
# (exit codes 0 = ok and 1 = test failures are the only ones that let it continue).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP_OK() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }

timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -5 gpurun_out/gpu_tests.log
STEP_OK $rc || exit $rc

BENCH_ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1"}
timeout -k 10 900 python bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc

if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
      python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.err
  find gpurun_out/prof -name '*stats*' | head
fi

#!/bin/bash
# One GPU session: parity tests, a bench line, a rocprofv3 kernel-trace summary, PMC passes.
#   STEPS="tests bench prof pmc list" TAG=v14 bash tools/session.sh
# Every GPU step runs under its own time limit and the session stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-"tests bench prof"}
TAG=${TAG:-cur}
BENCH_ARGS=${BENCH_ARGS:-"--steps 5 --warmup 1"}
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
          -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1
      rc=$?; echo "gpu tests rc=$rc"; tail -4 gpurun_out/${TAG}_gpu_tests.log ;;
    bench)
      timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
      rc=$?; echo "bench rc=$rc"; cut -c 1-400 gpurun_out/${TAG}_bench.json; tail -3 gpurun_out/${TAG}_bench.err ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
          python bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-drop-in > gpurun_out/${TAG}_prof_bench.json \
          2> gpurun_out/${TAG}_prof.err
      rc=$?; echo "rocprof rc=$rc" ;;
    pmc)
      PMC_NAME=${TAG}_c3 PMC_BENCH_ARGS="--config c3" bash tools/pmc.sh; rc=$? ;;
    list)
      timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; rc=$?; echo "list rc=$rc" ;;
    *) echo "unknown step $s"; rc=2 ;;
  esac
  [ $rc -eq 0 ] || exit $rc
done

#!/bin/bash
# One GPU session of round 6: parity tests, smoke, the C3 bench line (live PMC), C1 / C2 / C5 lines,
# and the one-GPU timing of the strong-scaled c3 shards (1024^2 @ 256/N spp, N = 2, 4, 8).
#   OUT=gpurun_out/r06a TESTS=1 bash tools/r06_check.sh
# Every GPU step has its own time limit and the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06}
mkdir -p "$O"
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
      > "$O/gpu_tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$O/gpu_tests.log"; exit 1; }
  tail -2 "$O/gpu_tests.log"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke rc=$?"; exit 1; }
  cat "$O/smoke.log"
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$O/bench_c3.json" 2> "$O/bench_c3.err" || { echo "bench rc=$?"; tail "$O/bench_c3.err"; exit 1; }
  echo bench ok
fi
if [ "${CONFIGS:-1}" = 1 ]; then
  for c in c1 c2; do
    timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-drop-in --no-pmc \
        > "$O/bench_$c.json" 2> "$O/bench_$c.err" || { echo "$c rc=$?"; exit 1; }
  done
  timeout -k 10 300 python bench.py --config c5 --steps 2 --no-cpu-baseline --no-drop-in > "$O/bench_c5.json" 2> "$O/bench_c5.err" || { echo "c5 rc=$?"; exit 1; }
  echo configs ok
fi
if [ "${SHARDS:-1}" = 1 ]; then
  # rank r's shard of the strong-scaled c3 frame at N = 8, 4, 2 GPUs, timed alone on this GPU
  for s in 32 64 128 256; do
    timeout -k 10 300 python bench.py --config c3 --spp $s --steps 20 --warmup 3 --no-cpu-baseline --no-drop-in --no-pmc \
        > "$O/shard_spp$s.json" 2> "$O/shard_spp$s.err" || { echo "shard $s rc=$?"; exit 1; }
  done
  echo shards ok
fi
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
      python3 bench.py --steps 5 --no-pmc --no-cpu-baseline --no-drop-in > "$O/rocprof_c3_bench.json" 2> "$O/rocprof.err" \
      || { echo "prof rc=$?"; exit 1; }
  echo prof ok
fi

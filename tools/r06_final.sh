#!/bin/bash
# Round-6 closing check on one MI355X: GPU tests, smoke, the default bench line (c3, live PMC, CPU
# baseline, drop-in), c1 / c2 / c5 lines, rocprofv3 kernel statistics of the c3 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06j}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/gpu_tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$O/gpu_tests.log"; exit 1; }
tail -1 "$O/gpu_tests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke rc=$?"; exit 1; }
cat "$O/smoke.log"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$O/bench_c3.json" 2> "$O/bench_c3.err" || { echo "bench rc=$?"; tail "$O/bench_c3.err"; exit 1; }
echo bench ok
for c in c1 c2; do
  timeout -k 10 300 python bench.py --config $c --steps 40 --warmup 4 --no-cpu-baseline --no-drop-in --no-pmc > "$O/bench_$c.json" 2> "$O/bench_$c.err" || { echo "$c rc=$?"; exit 1; }
done
timeout -k 10 300 python bench.py --config c5 --steps 2 --no-cpu-baseline --no-drop-in > "$O/bench_c5.json" 2> "$O/bench_c5.err" || { echo "c5 rc=$?"; exit 1; }
echo configs ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --steps 5 --no-pmc --no-cpu-baseline --no-drop-in > "$O/rocprof_c3_bench.json" 2> "$O/rocprof.err" || { echo "prof rc=$?"; exit 1; }
echo prof ok

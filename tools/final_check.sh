set -u
O=gpurun_out/r05p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
echo tests ok
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; exit 1; }
echo smoke ok
timeout -k 10 400 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench rc=$?"; exit 1; }
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --no-pmc --no-cpu-baseline --no-drop-in > $O/rocprof_c3_bench.json 2> $O/rocprof.err || { echo "prof rc=$?"; exit 1; }
echo prof ok
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 2 --no-cpu-baseline --no-drop-in --no-pmc > $O/bench_c2.json 2> $O/bench_c2.err || { echo "c2 rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --config c5 --steps 2 --no-cpu-baseline --no-drop-in > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --config c1 --steps 20 --warmup 2 --no-cpu-baseline --no-drop-in --no-pmc > $O/bench_c1.json 2> $O/bench_c1.err || { echo "c1 rc=$?"; exit 1; }
echo configs ok

#!/bin/bash
# C1 A/B (round-6 lone_walk with up to four owners vs abx/libbase.so), then the GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06c}
mkdir -p "$O"
export TMPDIR=/tmp
for r in 1 2; do
  for L in abx/libbase.so vanrijn_amd/lib/libvanrijn_amd.so; do
    VR_LIBRARY=$L timeout -k 10 300 python tools/c1_frames.py 40 > "$O/c1_$(basename $L .so)_$r.json" 2> "$O/c1.err" || { echo "c1 rc=$?"; tail "$O/c1.err"; exit 1; }
  done
done
echo c1 ok
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$O/gpu_tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$O/gpu_tests.log"; exit 1; }
tail -2 "$O/gpu_tests.log"
timeout -k 10 300 python bench.py --config c1 --steps 20 --warmup 3 --no-cpu-baseline --no-drop-in --no-pmc > "$O/bench_c1.json" 2> "$O/bench_c1.err" || { echo "bench c1 rc=$?"; exit 1; }
echo bench ok

#!/bin/bash
# octant copies of the 4-wide tree (abx/liboct.so) against HEAD (abx/libbase.so): GPU tests on the
# octant build, then interleaved per-process timings and record digests on C3, C5-sized, C2, C1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06oct}
mkdir -p "$O"
export TMPDIR=/tmp
VR_LIBRARY=abx/liboct.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/gpu_tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$O/gpu_tests.log"; exit 1; }
tail -1 "$O/gpu_tests.log"
for sc in "main 1024 256 3" "c5 2048 16 3" "main 512 64 5" "bench 256 16 9"; do
  for r in 1 2; do
    for lib in base oct; do
      VR_LIBRARY=abx/lib$lib.so timeout -k 10 300 python tools/lib_ab.py $sc >> "$O/ab.jsonl" 2>> "$O/err" || { echo rc=$?; tail "$O/err"; exit 1; }
    done
  done
done
cut -c1-220 "$O/ab.jsonl"

#!/bin/bash
# 16-bit traversal-stack entries: A/B against 32-bit on C3 / C2 / 1024^2 @32 (one process each), then the GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06x}
mkdir -p "$O"
export TMPDIR=/tmp
for a in "main 1024 256 5" "main 512 64 9" "main 1024 32 9"; do
  timeout -k 10 300 python tools/stack16_ab.py $a >> "$O/s16_ab.jsonl" 2> "$O/s16.err" || { echo "ab rc=$?"; tail "$O/s16.err"; exit 1; }
done
cat "$O/s16_ab.jsonl"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/gpu_tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$O/gpu_tests.log"; exit 1; }
tail -1 "$O/gpu_tests.log"

#!/bin/bash
# Round-2 session A: section-cycle breakdown of the current build, and the C4 / C5 per-rank
# shares on one GPU (bench lines + kernel-trace stats).  Each GPU step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/cycles.py 64 main > gpurun_out/cycles_main.json 2> gpurun_out/cycles_main.err
rc=$?; echo "cycles main rc=$rc"; cat gpurun_out/cycles_main.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/cycles.py 64 bench > gpurun_out/cycles_bench.json 2> gpurun_out/cycles_bench.err
rc=$?; echo "cycles bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --scene c5 --width 4096 --height 4096 --spp 32 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5_4096.json 2> gpurun_out/c5_4096.err
rc=$?; echo "c5 rc=$rc"; cat gpurun_out/c5_4096.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --scene main --width 2048 --height 2048 --spp 128 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c4_2048.json 2> gpurun_out/c4_2048.err
rc=$?; echo "c4 rc=$rc"; cat gpurun_out/c4_2048.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python bench.py --scene c5 --width 4096 --height 4096 --spp 32 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_c5.json 2> gpurun_out/prof_c5.err
rc=$?; echo "prof c5 rc=$rc"

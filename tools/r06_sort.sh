#!/bin/bash
# Ray reordering probe with the analysis build abx/libsplit.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06t}
mkdir -p "$O"
export TMPDIR=/tmp
VR_LIBRARY=abx/libsplit.so SPLIT_SORT=1 SPLIT_REPS=1 timeout -k 10 500 python tools/split_probe.py c5 4096 8 > "$O/sort_c5.jsonl" 2> "$O/sort_c5.err" || { echo "c5 rc=$?"; tail "$O/sort_c5.err"; exit 1; }
cat "$O/sort_c5.jsonl"
VR_LIBRARY=abx/libsplit.so SPLIT_SORT=1 SPLIT_REPS=1 timeout -k 10 500 python tools/split_probe.py main 1024 256 > "$O/sort_c3.jsonl" 2> "$O/sort_c3.err" || { echo "c3 rc=$?"; tail "$O/sort_c3.err"; exit 1; }
cat "$O/sort_c3.jsonl"
# the cooperative tail's per-phase profile on C1 (analysis build -DVR_COOP_PROF: vrcoop / vrwave lines on stderr)
VR_LIBRARY=abx/libcoopprof.so timeout -k 10 300 python tools/c1_frames.py 6 > "$O/coopprof_c1.json" 2> "$O/coopprof_c1.err" || { echo "coopprof rc=$?"; exit 1; }
grep -c vrcoop "$O/coopprof_c1.err"
# two streams on the small frames (C1, C2) at N = 1
for c in c1 c2; do
  for n in 1 2; do
    timeout -k 10 300 python bench.py --config $c --streams $n --steps 40 --warmup 4 --no-cpu-baseline --no-drop-in --no-pmc \
        > "$O/bench_${c}_s$n.json" 2> "$O/bench_${c}_s$n.err" || { echo "$c s$n rc=$?"; exit 1; }
  done
done
echo small frames ok

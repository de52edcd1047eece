#!/bin/bash
# The megakernel-split probe on one GPU (analysis build abx/libsplit.so): timings for C3 and C5, then
# one PMC pass over the C3 probe (SQ_WAIT_ANY, VALU activity of every TRACE configuration).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06s}
mkdir -p "$O"
export TMPDIR=/tmp
export VR_LIBRARY=abx/libsplit.so
timeout -k 10 400 python tools/split_probe.py main 1024 256 > "$O/split_c3.jsonl" 2> "$O/split_c3.err" || { echo "c3 rc=$?"; tail "$O/split_c3.err"; exit 1; }
cat "$O/split_c3.jsonl"
timeout -k 10 400 python tools/split_probe.py c5 4096 8 > "$O/split_c5.jsonl" 2> "$O/split_c5.err" || { echo "c5 rc=$?"; tail "$O/split_c5.err"; exit 1; }
cat "$O/split_c5.jsonl"
SPLIT_REPS=1 timeout -s KILL 400 rocprofv3 --kernel-trace --output-format csv -d "$O/pmc" -o run --pmc SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -- python3 tools/split_probe.py main 1024 256 > "$O/pmc_c3.jsonl" 2> "$O/pmc_c3.err" || { echo "pmc rc=$?"; tail "$O/pmc_c3.err"; exit 1; }
echo pmc ok
unset VR_LIBRARY
timeout -k 10 300 python tools/c1_frames.py 40 > "$O/c1_frames.json" 2> "$O/c1_frames.err" || { echo "c1 rc=$?"; exit 1; }
cat "$O/c1_frames.json" | cut -c1-400
for s in 64 128; do
  for n in 1 2; do
    timeout -k 10 300 python bench.py --config c3 --spp $s --streams $n --steps 20 --warmup 3 --no-cpu-baseline --no-drop-in --no-pmc \
        > "$O/shard_spp${s}_s$n.json" 2> "$O/shard_spp${s}_s$n.err" || { echo "shard $s rc=$?"; exit 1; }
  done
done
echo shards ok

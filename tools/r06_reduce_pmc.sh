#!/bin/bash
# PMC of the ordered reduce (accumulate_kernel) at C3: VALU activity, waits, HBM bytes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06r}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$O/p1" -o run --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -- python3 bench.py --pmc-child --config c3 > "$O/p1.out" 2> "$O/p1.err" || { echo "p1 rc=$?"; tail "$O/p1.err"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$O/p2" -o run --pmc FETCH_SIZE -- python3 bench.py --pmc-child --config c3 > "$O/p2.out" 2> "$O/p2.err" || { echo "p2 rc=$?"; tail "$O/p2.err"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$O/p3" -o run --pmc WRITE_SIZE SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 -- python3 bench.py --pmc-child --config c3 > "$O/p3.out" 2> "$O/p3.err" || { echo "p3 rc=$?"; tail "$O/p3.err"; exit 1; }
echo ok

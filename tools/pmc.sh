#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only beside --pmc, as the
# MI355X guide prescribes) over a short bench run.  Output: gpurun_out/pmc/<pass>/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
ARGS=${PMC_BENCH_ARGS:-"--steps 1 --warmup 0 --no-cpu-baseline"}
echo "$ARGS" > gpurun_out/pmc/args.txt
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1
echo "list rc=$?"
run_pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/$name -o run --pmc "$@" -- \
      python bench.py $ARGS > gpurun_out/pmc/$name.out 2> gpurun_out/pmc/$name.err
  local rc=$?
  echo "pass $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
run_pass fetch FETCH_SIZE
run_pass write WRITE_SIZE
run_pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run_pass tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
run_pass sq2 SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES
run_pass sq3 SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32

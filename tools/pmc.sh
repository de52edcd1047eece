#!/bin/bash
# PMC passes over one bench.py launch of the render kernel: one counter group per rocprofv3 run,
# --kernel-trace beside --pmc only (MI355X_MICROARCH.md), each pass under its own time limit.
#   PMC_NAME=c3 PMC_BENCH_ARGS="--config c3" bash tools/pmc.sh   -> gpurun_out/pmc/<name>/<pass>/
# tools/pmc_summary.py then folds the passes into profiles/pmc_records.json (read by bench.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
NAME=${PMC_NAME:-c3}
OUT=gpurun_out/pmc/$NAME
mkdir -p "$OUT"
ARGS="${PMC_BENCH_ARGS:-} --steps 1 --warmup 0 --no-cpu-baseline --no-drop-in"
echo "$ARGS" > "$OUT/args.txt"
sha256sum vanrijn_amd/lib/libvanrijn_amd.so | cut -d' ' -f1 > "$OUT/lib.sha256"  # the build profiled
run_pass() {
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name" -o run --pmc "$@" -- \
      python bench.py $ARGS > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "pass $NAME/$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run_pass fetch FETCH_SIZE
run_pass write WRITE_SIZE
run_pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run_pass tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
run_pass sq2 SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_WR
run_pass sq3 SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32
run_pass sq4 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32

#!/bin/bash
# One GPU session: parity tests, bench lines, rocprofv3 kernel-trace summaries, PMC passes.
#   STEPS="tests bench prof pmc bench:c5 prof:c5 pmc:c5 list" TAG=v15 bash tools/session.sh
# A step "name:cN" runs that step on bench.py --config cN (default c3).  Every GPU step runs under
# its own time limit and the session stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-"tests bench prof"}
TAG=${TAG:-cur}
BENCH_ARGS=${BENCH_ARGS:-"--steps 5 --warmup 1"}
sha256sum vanrijn_amd/lib/libvanrijn_amd.so > gpurun_out/${TAG}_lib.sha256
for s in $STEPS; do
  step=${s%%:*}; cfg=c3
  [ "$step" != "$s" ] && cfg=${s#*:}
  case $step in
    tests)
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
          -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1
      rc=$?; echo "gpu tests rc=$rc"; tail -4 gpurun_out/${TAG}_gpu_tests.log ;;
    smoke)
      timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/${TAG}_smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${TAG}_smoke.log ;;
    bench)
      if [ "$cfg" = c3 ]; then args="$BENCH_ARGS"; else args="--config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-drop-in"; fi
      timeout -k 10 600 python bench.py $args > gpurun_out/${TAG}_bench_$cfg.json 2> gpurun_out/${TAG}_bench_$cfg.err
      rc=$?; echo "bench $cfg rc=$rc"; cut -c 1-400 gpurun_out/${TAG}_bench_$cfg.json; tail -3 gpurun_out/${TAG}_bench_$cfg.err ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_$cfg -o run -- \
          python bench.py --config $cfg --steps 2 --warmup 0 --no-cpu-baseline --no-drop-in \
          > gpurun_out/${TAG}_prof_bench_$cfg.json 2> gpurun_out/${TAG}_prof_$cfg.err
      rc=$?; echo "rocprof $cfg rc=$rc" ;;
    pmc)
      PMC_NAME=${TAG}_$cfg PMC_BENCH_ARGS="--config $cfg" bash tools/pmc.sh; rc=$? ;;
    cycles)
      timeout -k 10 300 python tools/cycles.py 64 main > gpurun_out/${TAG}_cycles_main.json 2> gpurun_out/${TAG}_cycles.err
      rc=$?; echo "cycles rc=$rc" ;;
    tail)
      timeout -k 10 300 python tools/wg_tail.py 256 main > gpurun_out/${TAG}_tail_main.json 2> gpurun_out/${TAG}_tail.err
      rc=$?; echo "tail rc=$rc"; cat gpurun_out/${TAG}_tail_main.json ;;
    dropin)
      timeout -k 10 400 python tools/dropin.py 1024 32 > gpurun_out/${TAG}_dropin.json 2> gpurun_out/${TAG}_dropin.err
      rc=$?; echo "dropin rc=$rc"; tail -1 gpurun_out/${TAG}_dropin.json ;;
    dist)
      # bench.py under torch.distributed.run at world size 1: the RCCL group, barriers, the
      # records' dist.reduce and the max-over-ranks timing that the 8-GPU runs take
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
          --master-port 29517 bench.py --config $cfg --gpus 1 --steps 2 --warmup 1 --no-cpu-baseline --no-drop-in \
          > gpurun_out/${TAG}_dist_$cfg.json 2> gpurun_out/${TAG}_dist_$cfg.err
      rc=$?; echo "dist $cfg rc=$rc"; cut -c 1-300 gpurun_out/${TAG}_dist_$cfg.json; tail -3 gpurun_out/${TAG}_dist_$cfg.err ;;
    ab)
      # alternating-process A/B of the libraries in $AB_LIBS (tools/ab.sh; ROUNDS, SCENES)
      timeout -k 10 1200 bash tools/ab.sh $AB_LIBS > gpurun_out/${TAG}_ab.txt 2>&1
      rc=$?; echo "ab rc=$rc"; tail -20 gpurun_out/${TAG}_ab.txt; cp gpurun_out/ab_libs.jsonl gpurun_out/${TAG}_ab_libs.jsonl ;;
    benchab)
      # bench.py --config $cfg with each library of $AB_LIBS in turn, ROUNDS rounds (no PMC / CPU legs)
      : > gpurun_out/${TAG}_benchab_$cfg.jsonl
      for r in $(seq 1 ${ROUNDS:-3}); do
        for L in $AB_LIBS; do
          VR_LIBRARY=$L timeout -k 10 300 python bench.py --config $cfg --steps ${AB_STEPS:-10} --warmup 2 \
              --no-cpu-baseline --no-drop-in --no-pmc 2>> gpurun_out/${TAG}_benchab.err | \
              python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().split(chr(10))[-1]); print(json.dumps({'lib': '$L', 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_ms'], 'reduce_ms': d['roofline'].get('reduce_kernel_ms'), 'value': d['value']}))" \
              >> gpurun_out/${TAG}_benchab_$cfg.jsonl
          rc=$?; [ $rc -eq 0 ] || break 2
        done
      done
      echo "benchab $cfg rc=$rc"; cat gpurun_out/${TAG}_benchab_$cfg.jsonl ;;
    libtests)
      # the GPU tests against another build of the library (abx/lib$cfg.so, e.g. the VR_STAGE_GUARD build)
      VR_LIBRARY=abx/lib$cfg.so timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 \
          --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests_$cfg.log 2>&1
      rc=$?; echo "gpu tests ($cfg) rc=$rc"; tail -4 gpurun_out/${TAG}_gpu_tests_$cfg.log ;;
    culldebug)
      # tools/debug_cull_pf.py (cut tile, culled vs unculled, staging pre-filled) with abx/lib$cfg.so
      VR_LIBRARY=abx/lib$cfg.so timeout -k 10 300 python -u tools/debug_cull_pf.py > gpurun_out/${TAG}_culldebug_$cfg.log 2>&1
      rc=$?; echo "culldebug ($cfg) rc=$rc"; grep -E "differing|guard|->" gpurun_out/${TAG}_culldebug_$cfg.log | head -12 ;;
    list)
      timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; rc=$?; echo "list rc=$rc" ;;
    *) echo "unknown step $s"; rc=2 ;;
  esac
  [ $rc -eq 0 ] || exit $rc
done

#!/bin/bash
# Round-3 GPU session A: opcode issue costs, the -m gpu suite, the early-stop A/B (VR_EARLY_STOP)
# and the staging-store A/B (non-temporal vs plain, WRITE_SIZE per launch).  Every GPU step has
# its own time limit; the session stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03a
mkdir -p $O
sha256sum vanrijn_amd/lib/libvanrijn_amd.so abx/*.so > $O/libs.sha256
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }

timeout -k 10 180 tools/opcost 2048 > $O/opcost.json 2> $O/opcost.err; ok $? opcost
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; ok $rc gpu-tests
for sc in main:256 bench:32 c5:16; do
  timeout -k 10 400 python tools/variants.py --scene ${sc%%:*} --spp ${sc##*:} --reps 3 --variants 0 --thresholds 52 \
      --env VR_EARLY_STOP=1,0 >> $O/ab_early_stop.jsonl 2>> $O/variants.err; ok $? "early-stop A/B $sc"
done
for L in base plain; do
  VR_LIBRARY=abx/lib$L.so timeout -k 10 300 python tools/variants.py --scene main --spp 256 --reps 3 --variants 0 \
      --thresholds 52 | sed "s|^|$L |" >> $O/ab_stage.jsonl 2>> $O/variants.err; ok $? "stage A/B $L"
  VR_LIBRARY=abx/lib$L.so timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $O/pmc_write_$L -o run \
      --pmc WRITE_SIZE -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-drop-in \
      > $O/pmc_write_$L.out 2> $O/pmc_write_$L.err; ok $? "pmc write $L"
done
cat $O/ab_early_stop.jsonl $O/ab_stage.jsonl | cut -c 1-220

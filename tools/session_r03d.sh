#!/bin/bash
# Round-3 GPU session D: parity after the live-block compaction, its A/B against the previous
# build, the VR_LEAF_FEW sweep (eager leaf rounds when few lanes traverse) on C1 / 1 spp / C3 / C5,
# opcode diagnostics (cndmask forms, v_fmac_f64) and the default bench line with live PMC.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03d}
mkdir -p $O
sha256sum vanrijn_amd/lib/libvanrijn_amd.so abx/*.so > $O/libs.sha256
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }

timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; ok $rc gpu-tests
timeout -k 10 120 tools/opcost 2048 cndmask > $O/opcost_cndmask.json 2> $O/opcost.err; ok $? opcost-cndmask
timeout -k 10 120 tools/opcost 2048 fmac > $O/opcost_fmac.json 2>> $O/opcost.err; ok $? opcost-fmac
ROUNDS=3 timeout -k 10 900 bash tools/ab.sh abx/libbase.so vanrijn_amd/lib/libvanrijn_amd.so > $O/ab_compact.txt 2>&1
ok $? ab-compact; tail -4 $O/ab_compact.txt
for sc in bench:256:16 main:1024:1 main:1024:256 c5:1024:16; do
  IFS=: read -r scene size spp <<< "$sc"
  timeout -k 10 400 python tools/variants.py --scene $scene --size $size --spp $spp --reps 3 --variants 0 \
      --thresholds 52 --env VR_LEAF_FEW=0,2,4,8,16 >> $O/sweep_leaf_few.jsonl 2>> $O/variants.err; ok $? "sweep $sc"
done
cut -c 1-200 $O/sweep_leaf_few.jsonl
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
cut -c 1-300 $O/bench_default.json; tail -3 $O/bench_default.err; ok $rc bench

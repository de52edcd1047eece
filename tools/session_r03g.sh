#!/bin/bash
# Round-3 GPU session G: the cooperative tail (VR_COOP): parity first (the record variant's decision
# tests run it in every launch's tail; the NaN scene's rays walk whole trees), then the tail
# diagnostics and the A/B against a build without it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03g}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
VR_LIBRARY=abx/libwatch.so timeout -k 10 300 python -u -m pytest tests/test_gpu_build.py tests/test_gpu_parity.py -x -v -s \
    --timeout 100 --timeout-method thread -p no:cacheprovider > $O/watch_tests.log 2>&1; rc=$?
grep -m 20 "watchdog" $O/watch_tests.log; tail -3 $O/watch_tests.log; ok $rc watch-tests
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1; rc=$?; tail -5 $O/gpu_tests.log; ok $rc gpu-tests
for c in "bench 256 16" "main 1024 1" "main 512 64"; do
  timeout -k 10 300 python tools/tail.py $c >> $O/tail.jsonl 2>> $O/tail.err; ok $? "tail $c"
done
cut -c 1-330 $O/tail.jsonl
timeout -k 10 300 python tools/longpath.py bench 256 16 > $O/longpath.jsonl 2>> $O/longpath.err; ok $? longpath
cat $O/longpath.jsonl
SCENES="main:256 bench:32 c5:16" ROUNDS=3 timeout -k 10 900 bash tools/ab.sh abx/libbase.so \
    vanrijn_amd/lib/libvanrijn_amd.so > $O/ab_coop.txt 2>&1; ok $? ab; tail -7 $O/ab_coop.txt
for L in abx/libbase.so vanrijn_amd/lib/libvanrijn_amd.so; do
  for sc in bench:256:16 main:1024:1; do
    IFS=: read -r scene size spp <<< "$sc"
    VR_LIBRARY=$L timeout -k 10 300 python tools/variants.py --scene $scene --size $size --spp $spp --reps 5 \
        --variants 0 --thresholds 52 | sed "s|^|$(basename $L) |" >> $O/small_frames.jsonl 2>> $O/variants.err
    ok $? "small $sc"
  done
done
cut -c 1-220 $O/small_frames.jsonl

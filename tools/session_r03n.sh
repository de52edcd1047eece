#!/bin/bash
# Round-3 GPU session N: the call-context pool prefers contexts whose work has finished (so two
# streams' frames overlap): the concurrency / parity tests, then frames alternated over two
# streams vs one (tools/pipeline_probe.py) at C3, C2, C1 and a C5 slice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03n}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_concurrency.py tests/test_gpu_parity.py tests/test_gpu_dist_rehearsal.py \
    -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; ok $rc tests
for sc in main:1024:256:6 main:512:64:20 bench:256:16:20 c5:2048:16:6; do
  IFS=: read -r scene size spp frames <<< "$sc"
  timeout -k 10 300 python tools/pipeline_probe.py $scene $size $spp $frames >> $O/pipeline.jsonl 2>> $O/pipeline.err
  ok $? "probe $sc"
done
cat $O/pipeline.jsonl

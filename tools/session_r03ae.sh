#!/bin/bash
# Round-3 GPU session AE: the cooperative tail gated at 48 bounces: small-frame timings with it on /
# off (C1, main 1024^2 @1, C2), C1's per-wave tail, and the -m gpu suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03ae}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
timeout -k 10 300 python tools/variants.py --scene bench --size 256 --spp 16 --reps 9 --variants 0 --thresholds 52 \
    --env VR_COOP=0,2 > $O/c1.jsonl 2>> $O/var.err; ok $? c1
timeout -k 10 300 python tools/variants.py --scene main --size 1024 --spp 1 --reps 9 --variants 0 --thresholds 52 \
    --env VR_COOP=0,2 > $O/main1.jsonl 2>> $O/var.err; ok $? main1
timeout -k 10 300 python tools/variants.py --scene main --size 512 --spp 64 --reps 5 --variants 0 --thresholds 52 \
    --env VR_COOP=0,2 > $O/c2.jsonl 2>> $O/var.err; ok $? c2
cut -c 1-180 $O/c1.jsonl $O/main1.jsonl $O/c2.jsonl
timeout -k 10 300 python tools/tail.py bench 256 16 > $O/tail_c1.json 2> $O/tail.err; ok $? tail
python3 -c "
import json
d = json.load(open('$O/tail_c1.json'))
print('kernel', round(d['kernel_ms_median'], 3), 'wg_end', d['wg_end_ms'])
print('  slowest', d['slowest_waves'][:4]); print('  by long paths', d['waves_by_long_paths'])
"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1; rc=$?; tail -2 $O/gpu_tests.log; ok $rc gpu-tests

#!/bin/bash
# Round-3 GPU session AA: the two-owner cooperative tail (COOP instantiations on launches of at most
# 4 M pixel-samples): the -m gpu suite (its small tiles now run the COOP kernel), the per-wave tail of
# C1 with it on and off, and small-frame timings (C1, one 1024^2 sample) with VR_COOP=0 / 1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03aa}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; ok $rc gpu-tests
timeout -k 10 300 python tools/tail.py bench 256 16 > $O/tail_c1_coop.json 2> $O/tail.err; ok $? tail-coop
VR_COOP=0 timeout -k 10 300 python tools/tail.py bench 256 16 > $O/tail_c1_nocoop.json 2>> $O/tail.err; ok $? tail-nocoop
python3 -c "
import json
for n in ('coop', 'nocoop'):
    d = json.load(open('$O/tail_c1_%s.json' % n))
    print(n, 'kernel', round(d['kernel_ms_median'], 3), 'wg_end', d['wg_end_ms'])
    print('  slowest', d['slowest_waves'][:5])
    print('  by long paths', d['waves_by_long_paths'])
"
timeout -k 10 300 python tools/variants.py --scene bench --size 256 --spp 16 --reps 7 --variants 0 --thresholds 52 \
    --env VR_COOP=0,1 > $O/small_c1.jsonl 2>> $O/var.err; ok $? small-c1
timeout -k 10 300 python tools/variants.py --scene main --size 1024 --spp 1 --reps 7 --variants 0 --thresholds 52 \
    --env VR_COOP=0,1 > $O/small_main1.jsonl 2>> $O/var.err; ok $? small-main1
timeout -k 10 300 python tools/variants.py --scene main --size 512 --spp 64 --reps 5 --variants 0 --thresholds 52 \
    --env VR_COOP=0,1 > $O/c2.jsonl 2>> $O/var.err; ok $? c2
cut -c 1-260 $O/small_c1.jsonl $O/small_main1.jsonl $O/c2.jsonl

#!/bin/bash
# Round-3 GPU session AD: per-wave tail of main 1024^2 @1 with the cooperative tail on / off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03ad}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
for co in 2 0; do
  VR_COOP=$co timeout -k 10 300 python tools/tail.py main 1024 1 > $O/tail_main1_coop$co.json 2>> $O/tail.err; ok $? tail-$co
done
python3 -c "
import json
for co in (2, 0):
    d = json.load(open('$O/tail_main1_coop%d.json' % co))
    print(co, 'kernel', round(d['kernel_ms_median'], 3), 'wg_end', d['wg_end_ms'], d['bounces'])
    print('  slowest', d['slowest_waves'][:8])
"

#!/bin/bash
# Round-3 GPU session Z: which waves make C1's tail (benches/simple_scene.rs scene, 256^2 @16): per-wave
# end time, longest path and count of >= 64-bounce paths, for the default build and the cooperative-
# tail build (VR_COOP=1, a lone path's walk spread over its wave's lanes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03z}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
timeout -k 10 300 python tools/tail.py bench 256 16 > $O/tail_c1_default.json 2> $O/tail.err; ok $? tail-default
VR_LIBRARY=abx/libcoop.so VR_COOP=1 timeout -k 10 300 python tools/tail.py bench 256 16 > $O/tail_c1_coop.json 2>> $O/tail.err; ok $? tail-coop
python3 -c "
import json
for n in ('default', 'coop'):
    d = json.load(open('$O/tail_c1_%s.json' % n))
    print(n, 'kernel', round(d['kernel_ms_median'], 3), 'wg_end', d['wg_end_ms'])
    print('  slowest', d['slowest_waves'][:6])
    print('  by long paths', d['waves_by_long_paths'])
"

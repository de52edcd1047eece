#!/bin/bash
# Round-3 GPU session AK: which build reads stale staging on a cut tile: tools/debug_cull_pf.py on
# b38f898 and on b38f898 + the reduce-prefetch patch; the hardened cull test on the latter.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03ak}
mkdir -p $O
for L in abx/lib_b38f898.so abx/lib_pf.so; do
  echo "== $L"; VR_LIBRARY=$L timeout -k 10 120 python tools/debug_cull_pf.py 2>&1 | grep "differing" || exit 1
done
VR_LIBRARY=abx/lib_pf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_cull.py -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > $O/cull_pf.log 2>&1; echo "pf build cull test rc=$? (expected failures)"; tail -2 $O/cull_pf.log
exit 0

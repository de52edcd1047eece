#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for L in abx/lib_8edc668.so abx/lib_74aa6be.so abx/lib_31bf95a.so; do
  echo "== $L"; VR_LIBRARY=$L timeout -k 10 120 python tools/debug_cull_pf.py 2>&1 | grep -v "amdgpu.ids\|__del__\|Traceback\|NoneType\|scene.py" | cut -c 1-200 || exit 1
done

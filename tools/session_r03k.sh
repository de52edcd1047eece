#!/bin/bash
# Round-3 GPU session K: LDS copy of the tree's top (VR_HOT_MAX): parity of the hot build, the A/B
# against HEAD and the no-LDS build of the same source, then a PC-sampling run of the -g build
# (dynamic instruction mix per source line: tools/pc_sections.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03k}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
VR_LIBRARY=abx/libhot32.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullframe.py \
    tests/test_gpu_build.py tests/test_gpu_cull.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > $O/hot_tests.log 2>&1
rc=$?; tail -3 $O/hot_tests.log; ok $rc hot-tests
SCENES="main:256 bench:32 c5:16" ROUNDS=3 timeout -k 10 1000 bash tools/ab.sh abx/libhead.so abx/libhot0.so \
    abx/libhot32.so abx/libhot16.so > $O/ab_hot.txt 2>&1; ok $? ab; tail -12 $O/ab_hot.txt
cp gpurun_out/ab_libs.jsonl $O/ab_hot.jsonl
timeout -k 10 60 rocprofv3 -L > $O/rocprof_list.txt 2>&1; echo "list rc=$?"
grep -i -A12 'pc.sampl' $O/rocprof_list.txt | head -40 || true
VR_LIBRARY=abx/libprof.so timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic \
    --pc-sampling-unit cycles --pc-sampling-interval 1048576 --output-format csv -d $O/pcs -o run -- \
    python tools/pcsample.py 64 main > $O/pcs.out 2> $O/pcs.err
echo "pc-sampling stochastic rc=$?"; tail -5 $O/pcs.err; ls -la $O/pcs 2>/dev/null | head

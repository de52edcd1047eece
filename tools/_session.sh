set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc

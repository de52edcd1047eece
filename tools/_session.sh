set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python tools/variants.py --spp 32 --reps 3 --variants 0,1,2,3,4 --thresholds 32 > gpurun_out/variants.jsonl 2> gpurun_out/variants.err
rc=$?; echo "variants rc=$rc"; cat gpurun_out/variants.jsonl; tail -3 gpurun_out/variants.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/variants.py --spp 32 --reps 2 --variants 0 --thresholds 0,8,16,24,40,48,56 > gpurun_out/thresholds.jsonl 2>> gpurun_out/variants.err
rc=$?; echo "thresholds rc=$rc"; cat gpurun_out/thresholds.jsonl

set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -25 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/variants.py --scene main --spp 256 --reps 2 --variants 0 --thresholds 56 > gpurun_out/ab.jsonl 2>> gpurun_out/variants.err
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/variants.py --scene bench --spp 32 --reps 3 --variants 0 --thresholds 56 >> gpurun_out/ab.jsonl 2>> gpurun_out/variants.err
rc=$?; echo "rc=$rc"; cut -c 1-190 gpurun_out/ab.jsonl

set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python tools/variants.py --spp 32 --reps 3 --variants 0,1,2,4 --thresholds 56 > gpurun_out/variants.jsonl 2> gpurun_out/variants.err
rc=$?; echo "var rc=$rc"; cat gpurun_out/variants.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/variants.py --scene bench --spp 32 --reps 3 --variants 0,1,2 --thresholds 56 > gpurun_out/variants_bench.jsonl 2>> gpurun_out/variants.err
rc=$?; echo "var bench rc=$rc"; cat gpurun_out/variants_bench.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json

set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python bench.py --scene c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5.json 2> gpurun_out/c5.err
rc=$?; echo "rc=$rc"; cat gpurun_out/c5.json; tail -3 gpurun_out/c5.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/variants.py --scene materials --spp 64 --reps 2 --variants 0 --thresholds 56 > gpurun_out/ab.jsonl 2>> gpurun_out/variants.err
timeout -k 10 600 python tools/variants.py --scene whitted --spp 64 --reps 2 --variants 0 --thresholds 56 >> gpurun_out/ab.jsonl 2>> gpurun_out/variants.err
rc=$?; echo "rc=$rc"; cut -c 1-200 gpurun_out/ab.jsonl

set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python tools/variants.py --scene bench --spp 32 --reps 2 --variants 0,1 --thresholds 56 --env VR_FORCE_MATS=2,3 > gpurun_out/mats.jsonl 2> gpurun_out/variants.err
rc=$?; echo "rc=$rc"; cat gpurun_out/mats.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/wg_tail.py 32 bench > gpurun_out/wg_tail.json 2> gpurun_out/wg_tail.err
rc=$?; echo "wg rc=$rc"; cat gpurun_out/wg_tail.json

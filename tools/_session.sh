set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python tools/variants.py --scene bench --spp 32 --reps 2 --variants 0 --thresholds 56 --env VR_CHUNK=1 --env VR_GRAB=256,512,1024,4096 >> gpurun_out/grab2.jsonl 2>> gpurun_out/variants.err
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { cat gpurun_out/grab2.jsonl; exit $rc; }
timeout -k 10 700 python tools/variants.py --scene main --spp 256 --reps 2 --variants 0 --thresholds 40,56 --env VR_CHUNK=1 --env VR_GRAB=256,512,1024,4096 --env VR_PHASE_A_REPS=1,2 >> gpurun_out/grab2.jsonl 2>> gpurun_out/variants.err
rc=$?; echo "rc=$rc"; cut -c 1-180 gpurun_out/grab2.jsonl

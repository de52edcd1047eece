#!/bin/bash
# bench.py's N = 4 and N = 8 paths rehearsed on one GPU at C3's full size (all ranks on cuda:0, the
# records reduced through gloo on host copies): the rank-count-dependent splits end to end
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06reh}
mkdir -p "$O"
export TMPDIR=/tmp
for n in 4 8; do
  timeout -k 10 500 python bench.py --gpus $n --one-gpu-rehearsal --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-drop-in > "$O/reh$n.json" 2> "$O/reh$n.err" || { echo "n=$n rc=$?"; tail -20 "$O/reh$n.err"; exit 1; }
  echo "n=$n ok"; cut -c1-400 "$O/reh$n.json"
done

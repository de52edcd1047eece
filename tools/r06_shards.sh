#!/bin/bash
# the strong-scaled c3 shards on one GPU (1024^2 @ 256/N spp), default streams per N, same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06sh}
mkdir -p "$O"
export TMPDIR=/tmp
for s in 256 128 64 32; do
  n=1; [ $s -lt 256 ] && n=2
  timeout -k 10 300 python bench.py --config c3 --spp $s --streams $n --steps 20 --warmup 3 --no-cpu-baseline --no-drop-in --no-pmc > "$O/shard_spp${s}.json" 2> "$O/shard_spp${s}.err" || { echo "shard $s rc=$?"; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/shard_spp${s}.json').read().strip().splitlines()[-1]);print($s, d['ms_per_step'], d['config']['streams'], d.get('sequential',{}).get('ms_per_step'))"
done

#!/bin/bash
# the N = 2 shard of c3 (1024^2 @128) with one and two streams, interleaved, three times each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06st128}
mkdir -p "$O"
export TMPDIR=/tmp
for r in 1 2 3; do
  for n in 1 2; do
    timeout -k 10 300 python bench.py --config c3 --spp 128 --streams $n --steps 30 --warmup 3 --no-cpu-baseline --no-drop-in --no-pmc > "$O/s${n}_r$r.json" 2>> "$O/err" || { echo "rc=$?"; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/s${n}_r$r.json').read().strip().splitlines()[-1]);print('streams', $n, 'round', $r, d['ms_per_step'], d.get('sequential',{}).get('ms_per_step'))"
  done
done

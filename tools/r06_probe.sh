#!/bin/bash
# Round-6 probes on one GPU: frame pipelining over two streams, guided queue slices (tuning build
# abx/libtune.so: VR_TAPER), the COOP grid (VR_COOP_GRID), and the launch tail at 32 spp.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r06p}
mkdir -p "$O"
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 300 "$@" > "$O/$name.out" 2> "$O/$name.err" || { echo "$name rc=$?"; tail -5 "$O/$name.err"; exit 1; }; echo "$name ok"; }
T=abx/libtune.so
run taper32 env VR_LIBRARY=$T python tools/variants.py --spp 32 --reps 7 --variants 0 --thresholds 52 --env VR_TAPER=0,1
run taper256 env VR_LIBRARY=$T python tools/variants.py --spp 256 --reps 3 --variants 0 --thresholds 52 --env VR_TAPER=0,1
run taper_c2 env VR_LIBRARY=$T python tools/variants.py --spp 64 --size 512 --reps 5 --variants 0 --thresholds 52 --env VR_TAPER=0,1
run coopgrid env VR_LIBRARY=$T python tools/variants.py --scene bench --size 256 --spp 16 --reps 9 --variants 0 --thresholds 52 --env VR_COOP_GRID=2,3 --env VR_TAPER=0,1
run tail32_on env VR_LIBRARY=$T VR_TAPER=1 python tools/wg_tail.py 32 main
run tail32_off env VR_LIBRARY=$T VR_TAPER=0 python tools/wg_tail.py 32 main
run pipe32 python tools/pipeline_probe.py main 1024 32 20
run pipe256 python tools/pipeline_probe.py main 1024 256 6
for s in 1 2; do
  run bench32_s$s python bench.py --config c3 --spp 32 --streams $s --steps 40 --warmup 4 --no-cpu-baseline --no-drop-in --no-pmc
  run bench256_s$s python bench.py --config c3 --streams $s --steps 10 --warmup 2 --no-cpu-baseline --no-drop-in --no-pmc
done

#!/bin/bash
# Round-3 GPU session AB: why the two-owner cooperative tail slows the main scene's small frames:
# counters of main 1024^2 @1 with VR_COOP = 0 / 1 / 2, and the timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03ab}
mkdir -p $O
ok() { local rc=$1; shift; echo "$* rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
timeout -k 10 300 python - > $O/counts_main1.jsonl 2> $O/counts.err <<'PY'
import json, os, sys, torch
sys.path.insert(0, os.getcwd())
from vanrijn_amd import scenes
from vanrijn_amd.render import Tile, render_tile_device
for name, sc, size, spp in (("main", scenes.main_scene(), 1024, 1), ("bench", scenes.bench_scene(), 256, 16)):
    ds = sc.device_scene(0)
    st = torch.zeros(size * size * 8, dtype=torch.float64, device="cuda")
    for co in ("0", "2"):
        os.environ["VR_COOP"] = co
        t = [render_tile_device(ds, Tile(0, size, 0, size), size, size, spp, 1, 0, st.data_ptr(),
                                torch.cuda.current_stream().cuda_stream, timed=True)["kernel_ms"] for _ in range(5)]
        c = render_tile_device(ds, Tile(0, size, 0, size), size, size, spp, 1, 0, st.data_ptr(),
                               torch.cuda.current_stream().cuda_stream, counters=True)
        print(json.dumps({"scene": name, "coop": co, "timed_ms": sorted(t)[2], **{k: c[k] for k in (
            "node_visits", "box_tests", "triangle_tests", "rays", "traversal_slots", "path_loop_slots", "kernel_ms")}}), flush=True)
PY
ok $? counts
cat $O/counts_main1.jsonl | cut -c 1-330
timeout -k 10 300 python tools/variants.py --scene main --size 512 --spp 64 --reps 5 --variants 0 --thresholds 52 \
    --env VR_COOP=0,2 > $O/c2.jsonl 2>> $O/var.err; ok $? c2
timeout -k 10 300 python tools/variants.py --scene bench --size 256 --spp 16 --reps 7 --variants 0 --thresholds 52 \
    --env VR_COOP=0,2 > $O/c1.jsonl 2>> $O/var.err; ok $? c1
cut -c 1-200 $O/c2.jsonl $O/c1.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1; rc=$?; tail -2 $O/gpu_tests.log; ok $rc gpu-tests

"""One warm render of the bench configuration for PC sampling / ISA attribution runs:
    rocprofv3 --pc-sampling-beta-enabled ... -- python tools/pcsample.py [spp] [scene]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vanrijn_amd import scenes  # noqa: E402
from vanrijn_amd.render import Tile, render_tile_device  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
which = sys.argv[2] if len(sys.argv) > 2 else "main"
torch.cuda.set_device(0)
ds = (scenes.main_scene() if which == "main" else scenes.bench_scene()).device_scene(0)
state = torch.zeros(1024 * 1024 * 8, dtype=torch.float64, device="cuda")
for i in range(2):
    st = render_tile_device(ds, Tile(0, 1024, 0, 1024), 1024, 1024, spp, 1, i * spp, state.data_ptr(),
                            torch.cuda.current_stream().cuda_stream, timed=True)
    print(i, st["kernel_ms"], flush=True)

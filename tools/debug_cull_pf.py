"""Debug: tests/test_gpu_cull.py's cut tile, culled vs unculled records, with the library in VR_LIBRARY:
where they differ."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vanrijn_amd import records as R  # noqa: E402
from vanrijn_amd import scenes  # noqa: E402
from vanrijn_amd.render import Tile, render_tile_device, stream_check_error  # noqa: E402

ds = scenes.main_scene().device_scene(0)
t = Tile(5, 203, 100, 300)
H, W = 300, 400
npix = (t.end_column - t.start_column) * (t.end_row - t.start_row)
stream = torch.cuda.current_stream().cuda_stream


def run(cull, stages):
    st = torch.zeros(npix * 8, dtype=torch.float64, device="cuda")
    for spp, first, acc in stages:
        render_tile_device(ds, t, H, W, spp, 0x77, first, st.data_ptr(), stream, accumulate=acc, cull=cull)
    torch.cuda.synchronize()
    try:
        stream_check_error(ds, stream)  # a guard build's stale-staging report, if any
    except Exception as e:  # noqa: BLE001
        print("  cull" if cull else "  no cull", stages, "->", e)
    st = st.cpu()
    return torch.cat([R.sums(st), R.compensations(st)], dim=1)  # [pixel][8]


# first, other photons into the call contexts' staging (every sample traced, another seed)
junk = torch.zeros(npix * 8, dtype=torch.float64, device="cuda")
for k in range(2):
    render_tile_device(ds, t, H, W, 4, 0x1234 + k, 0, junk.data_ptr(), stream, cull=False)
for stages in ([(4, 0, False)], [(4, 0, False), (3, 4, True)], [(4, 0, False), (3, 4, True), (2, 7, True)]):
    a, b = run(False, stages), run(True, stages)
    d = (a != b).any(dim=1).nonzero().reshape(-1)
    print(stages, "differing pixels", len(d))
    for i in d[:4].tolist():
        print("  pixel", i, "row", i // 198, "col", i % 198, "nocull", a[i].tolist(), "cull", b[i].tolist())

"""Debug: the 'ties' mesh (vertices on a half-integer grid) rendered through the SAH host tree,
the reference host tree and the device-built tree, against the oracle's reference mode."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa
from vanrijn_amd.render import Tile, render_samples
from vanrijn_amd.scene import LambertianMaterial, Mesh, Scene, Spectrum, BoundingVolumeHierarchy
from oracle import oracle_ffi as O

rng = np.random.default_rng(11)
v = np.round(rng.normal(size=(3000, 3, 3)) * 2) / 2
n = np.zeros_like(v); n[..., 2] = 1.0
sc = Scene((0.0, 0.0, -5.0), [BoundingVolumeHierarchy.build(Mesh(v, n, LambertianMaterial(Spectrum.grey(0.5), 0.5)))])
W, H = 48, 40
t = Tile(0, W, 0, H)
orc = O.OracleScene(sc.spec())
ref = orc.render_samples(t, H, W, 3, seed=0x5EED0001, mode=O.MODE_REFERENCE, nthreads=8)
res = {}
for name, kw in (("sah", {}), ("refbvh", {"reference_bvh": True}), ("device", {"device_bvh": True})):
    ds = sc.device_scene(0, **kw)
    g = render_samples(ds, t, H, W, 3, seed=0x5EED0001)
    res[name] = g
    bad = np.flatnonzero((g["flags"] != ref["flags"]).ravel() | (g["bounces"] != ref["bounces"]).ravel())
    print(name, "differs from oracle in", len(bad), "of", g["flags"].size, "samples; first", bad[:8])

# the differing samples: camera-ray traces through each tree vs the oracle
for name in res:
    g = res[name]
    d = np.argwhere((g["flags"] != ref["flags"]) | (g["bounces"] != ref["bounces"]))
    for (y, x, k) in d[:3]:
        print(name, "pixel", (y, x), "sample", k, "gpu flags/bounces", g["flags"][y, x, k], g["bounces"][y, x, k],
              "oracle", ref["flags"][y, x, k], ref["bounces"][y, x, k], "wl", g["wavelength"][y, x, k], ref["wavelength"][y, x, k])

for name in res:
    g = res[name]
    di = np.abs(g["intensity"] - ref["intensity"])
    print(name, "max |dI| vs oracle", di.max(), "n differing", int((g["intensity"] != ref["intensity"]).sum()),
          "wl differ", int((g["wavelength"] != ref["wavelength"]).sum()))
a, b = res["sah"], res["device"]
dd = np.argwhere(a["intensity"] != b["intensity"])
print("sah vs device intensity differ:", len(dd), dd[:5])
for (y, x, k) in dd[:3]:
    print((y, x, k), a["intensity"][y, x, k], b["intensity"][y, x, k], ref["intensity"][y, x, k], a["bounces"][y, x, k])
# accumulation through render_tile_device
from vanrijn_amd import records as R  # noqa: E402
from vanrijn_amd.render import render_tile_device
outs = {}
for name, kw in (("sah", {}), ("device", {"device_bvh": True})):
    ds = sc.device_scene(0, **kw)
    st = torch.zeros(H * W * 8, dtype=torch.float64, device="cuda")
    render_tile_device(ds, t, H, W, 3, 0x5EED0001, 0, st.data_ptr())
    f = R.fields(st)  # per pixel: colour_sum, colour_bias, weight, weight_bias side by side
    outs[name] = np.concatenate([f["colour_sum"], f["colour_bias"], f["weight"][:, None],
                                 f["weight_bias"][:, None]], axis=1).reshape(H, W, 8)
dz = np.argwhere(outs["sah"] != outs["device"])
print("records differ at", len(dz), dz[:6])
for (y, x, c) in dz[:4]:
    print((y, x, c), outs["sah"][y, x], outs["device"][y, x])

"""Debug: the 'ties' scene's differing samples rendered alone (tiny tiles), against the oracle, to tell
a decision that depends on a sample's wave-mates from one that does not."""
import os, sys
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
orc = O.OracleScene(sc.spec())
ref = orc.render_samples(Tile(0, W, 0, H), H, W, 3, seed=0x5EED0001, mode=O.MODE_REFERENCE, nthreads=8)
ds = sc.device_scene(0)
full = render_samples(ds, Tile(0, W, 0, H), H, W, 3, seed=0x5EED0001)
bad = np.argwhere(full["bounces"] != ref["bounces"])
print("full-tile differing samples:", len(bad))
for (y, x, k) in bad[:12]:
    one = render_samples(ds, Tile(int(x), int(x) + 1, int(y), int(y) + 1), H, W, 3, seed=0x5EED0001)
    row = render_samples(ds, Tile(0, W, int(y), int(y) + 1), H, W, 3, seed=0x5EED0001)
    print((int(y), int(x), int(k)), "oracle", ref["bounces"][y, x, k], "full", full["bounces"][y, x, k],
          "alone", one["bounces"][0, 0, k], "row", row["bounces"][0, x, k])

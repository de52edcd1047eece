"""Scene-build time of the C5 synthetic mesh (1,051,392 triangles): host vs device BVH build.
    python tools/build_timing.py"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vanrijn_amd import scenes  # noqa: E402
from vanrijn_amd.scene import BoundingVolumeHierarchy, LambertianMaterial, Mesh, Scene, Spectrum  # noqa: E402

import torch  # noqa: E402,F401  (binds the HIP runtime first, as bench.py does)

v, n = scenes.synthetic_sphere_mesh()
out = {"triangles": int(len(v))}
for name, kw in (("device", dict(device_bvh=True)), ("host", dict()), ("device_again", dict(device_bvh=True))):
    s = Scene(scenes.CAMERA_LOCATION, [BoundingVolumeHierarchy.build(Mesh(v, n, LambertianMaterial(Spectrum.grey(0.5),
                                                                                                     0.5)))])
    t0 = time.perf_counter()
    ds = s.device_scene(0, **kw)
    out[f"{name}_s"] = round(time.perf_counter() - t0, 3)
    out[f"{name}_depth"] = ds.info()["max_bvh_depth"]
print(json.dumps(out))

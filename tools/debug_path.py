"""Debug: one sample of the 'ties' scene (tools/debug_ties.py) rendered by a VR_DEBUG_PIX / VR_DEBUG_SMP
build of the render kernel, which prints every traced ray and its closest hit; each ray is then traced
by the oracle (reference mode) and the first disagreement printed.
    VR_LIBRARY=abx/libdbg.so python tools/debug_path.py   (pixel / sample compiled into the library)"""
import os, subprocess, sys, struct
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r'''
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from vanrijn_amd.render import Tile, render_samples
from vanrijn_amd.scene import LambertianMaterial, Mesh, Scene, Spectrum, BoundingVolumeHierarchy
rng = np.random.default_rng(11)
v = np.round(rng.normal(size=(3000, 3, 3)) * 2) / 2
n = np.zeros_like(v); n[..., 2] = 1.0
sc = Scene((0.0, 0.0, -5.0), [BoundingVolumeHierarchy.build(Mesh(v, n, LambertianMaterial(Spectrum.grey(0.5), 0.5)))])
g = render_samples(sc.device_scene(0), Tile(0, 48, 0, 40), 40, 48, 3, seed=0x5EED0001)
torch.cuda.synchronize()
'''


def f(h):
    return struct.unpack("<d", struct.pack("<Q", int(h, 16)))[0]


def main():
    out = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, timeout=300)
    lines = [l.split() for l in out.stdout.splitlines() if l.startswith("vrdbg")]
    print("gpu rays:", len(lines), out.stderr[-300:] if out.returncode else "")
    from oracle import oracle_ffi as O
    from vanrijn_amd.scene import LambertianMaterial, Mesh, Scene, Spectrum, BoundingVolumeHierarchy
    rng = np.random.default_rng(11)
    v = np.round(rng.normal(size=(3000, 3, 3)) * 2) / 2
    n = np.zeros_like(v); n[..., 2] = 1.0
    sc = Scene((0.0, 0.0, -5.0), [BoundingVolumeHierarchy.build(Mesh(v, n, LambertianMaterial(Spectrum.grey(0.5), 0.5)))])
    orc = O.OracleScene(sc.spec())
    for l in lines:
        depth, kind, idx = int(l[1]), int(l[2]), int(l[3])
        d = f(l[4]); o = [f(x) for x in l[5:8]]; dr = [f(x) for x in l[8:11]]; rank = int(l[11])
        hits, _ = orc.trace([o], [dr])
        h = O.hit_to_dict(hits[0])
        od = h["distance"] if h else None
        same = (h is None and kind == 0) or (h is not None and kind != 0 and od == d)
        print(depth, "gpu", kind, rank, repr(d), "oracle", (h["primitive"], repr(od)) if h else None, "OK" if same else "DIFF",
              "o", o, "d", dr)
        if not same:
            break


if __name__ == "__main__":
    main()

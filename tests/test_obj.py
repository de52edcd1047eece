"""mesh::load_obj (src/mesh.rs:13-88) over the obj 0.9 crate: the library's C++ loader against an
independent Python restatement of the same rules.

Rules (mesh.rs + obj 0.9's parser; the crate's source is not in the container, so parity with
the crate itself is unpinned -- no reference test covers the loader):
  * `v x y z [w]` / `vn x y z`: f32 parses (correctly rounded), widened to f64 (mesh.rs:21-36);
  * `f` corners `v`, `v/t`, `v//n`, `v/t/n`: 1-based, negative = relative to the elements read so
    far; texture indices unused but validated;
  * polygons fan-triangulate as (v0, v_i, v_{i+1}) (mesh.rs:43-72); < 3 corners -> nothing;
  * a corner without a normal gets (0, 0, 0) (mesh.rs:30-37);
  * objects / groups flatten in file order (mesh.rs:82-85); other statements carry no geometry;
  * malformed numbers or out-of-range indices are I/O errors (load_obj returns io::Result).
"""
import numpy as np
import pytest

from vanrijn_amd import _native as N
from vanrijn_amd import scenes
from vanrijn_amd.scene import load_obj


def py_load_obj(text):
    pos, nrm, ntex, vs, ns = [], [], 0, [], []

    def res(i, n):
        return i - 1 if i > 0 else n + i

    for line in text.splitlines():
        t = line.split("#", 1)[0].split()
        if not t:
            continue
        if t[0] == "v":
            pos.append([float(np.float32(x)) for x in t[1:4]])
        elif t[0] == "vn":
            nrm.append([float(np.float32(x)) for x in t[1:4]])
        elif t[0] == "vt":
            ntex += 1
        elif t[0] == "f":
            corners = []
            for c in t[1:]:
                parts = c.split("/")
                v = res(int(parts[0]), len(pos))
                n = res(int(parts[2]), len(nrm)) if len(parts) == 3 and parts[2] else None
                corners.append((v, n))
            for i in range(1, len(corners) - 1):
                tri = [corners[0], corners[i], corners[i + 1]]
                vs.append([pos[v] for v, _ in tri])
                ns.append([nrm[n] if n is not None else [0.0, 0.0, 0.0] for _, n in tri])
    return np.array(vs, dtype=np.float64).reshape(-1, 3, 3), np.array(ns, dtype=np.float64).reshape(-1, 3, 3)


def random_obj(rng, n_v=40, n_n=25, n_t=10, n_f=60):
    lines = ["# generated", "mtllib x.mtl", "o first", "g group_a", "s 1"]
    nv = nn = nt = 0

    def num():
        k = rng.integers(4)
        x = rng.normal() * 10.0 ** int(rng.integers(-3, 4))
        return [f"{x:.9g}", f"{x:e}", f"{x:+.3f}", repr(float(np.float32(x)))][k]

    for _ in range(n_v):
        lines.append("v " + " ".join(num() for _ in range(3)) + (" 1.0" if rng.random() < 0.1 else ""))
        nv += 1
    for _ in range(n_t):
        lines.append(f"vt {rng.random():.4f} {rng.random():.4f}")
        nt += 1
    for _ in range(n_n):
        lines.append("vn " + " ".join(num() for _ in range(3)))
        nn += 1
    for f in range(n_f):
        if f == n_f // 2:
            lines += ["o second", "g group_b", "usemtl m", ""]
        k = int(rng.integers(3, 7))
        style = int(rng.integers(4))
        corners = []
        for _ in range(k):
            vi = int(rng.integers(1, nv + 1))
            vi = vi if rng.random() < 0.7 else vi - nv - 1  # negative = relative
            ti = int(rng.integers(1, nt + 1))
            ni = int(rng.integers(1, nn + 1))
            ni = ni if rng.random() < 0.7 else ni - nn - 1
            corners.append([f"{vi}", f"{vi}/{ti}", f"{vi}//{ni}", f"{vi}/{ti}/{ni}"][style])
        lines.append("f " + " ".join(corners) + ("  # trailing comment" if rng.random() < 0.1 else ""))
    return "\r\n".join(lines) + "\n" if rng.random() < 0.5 else "\n".join(lines) + "\n"


@pytest.mark.parametrize("seed", range(6))
def test_loader_matches_restatement(tmp_path, seed):
    rng = np.random.default_rng(seed)
    text = random_obj(rng)
    p = tmp_path / "m.obj"
    p.write_bytes(text.encode())
    m = load_obj(p, None)
    v, n = py_load_obj(text)
    assert m.vertices.shape == v.shape and np.array_equal(m.vertices, v)
    assert np.array_equal(m.normals, n)


def test_loader_polygon_and_degenerate_faces(tmp_path):
    p = tmp_path / "poly.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nv 0.5 1.5 0\nf 1 2\nf 1\nf 1 2 3 4 5\n")
    m = load_obj(p, None)
    assert m.vertices.shape == (3, 3, 3)  # the 2- and 1-corner faces yield nothing; pentagon -> 3
    assert np.array_equal(m.vertices[2], [[0, 0, 0], [0, 1, 0], [0.5, 1.5, 0]])


@pytest.mark.parametrize("body", ["v 0 0 zero\nf 1 1 1\n", "v 0 0 0\nf 1 2 3\n", "v 0 0 0\nf 0 1 1\n",
                                  "v 0 0 0\nvn 0 0 1\nf 1//2 1//1 1//1\n", "v 0 0 0\nf 1/5 1 1\n",
                                  "v 0 0 0\nf 1x 1 1\n", "vn 1 2\n"])
def test_loader_rejects_malformed(tmp_path, body):
    p = tmp_path / "bad.obj"
    p.write_text(body)
    with pytest.raises(N.VrError) as e:
        load_obj(p, None)
    assert e.value.code == -6


def test_procedural_bunny_obj_roundtrip(tmp_path):
    v, n = scenes.procedural_bunny()
    v32, n32 = v.astype(np.float32), n.astype(np.float32)
    lines = []
    for t in range(len(v)):
        for k in range(3):
            lines.append("v %s %s %s" % tuple(repr(float(x)) for x in v32[t, k]))
            lines.append("vn %s %s %s" % tuple(repr(float(x)) for x in n32[t, k]))
        b = 3 * t + 1
        lines.append(f"f {b}//{b} {b + 1}//{b + 1} {b + 2}//{b + 2}")
    p = tmp_path / "bunny.obj"
    p.write_text("\n".join(lines) + "\n")
    m = load_obj(p, None)
    assert np.array_equal(m.vertices, v32.astype(np.float64))
    assert np.array_equal(m.normals, n32.astype(np.float64))


def test_load_bunny_rejects_a_different_file(tmp_path):
    p = tmp_path / "stanford_bunny.obj"
    p.write_text("v 0 0 0\n")
    with pytest.raises(ValueError):
        scenes.load_bunny(str(p))


@pytest.mark.gpu
def test_obj_mesh_renders_like_the_oracle(tmp_path, oracle):
    """A loaded OBJ mesh (f32-rounded procedural bunny) through the GPU path vs the oracle."""
    from vanrijn_amd.render import Tile, render_samples
    v, n = scenes.procedural_bunny()
    lines = []
    for t in range(len(v)):
        for k in range(3):
            lines.append("v %s %s %s" % tuple(repr(float(x)) for x in v[t, k].astype(np.float32)))
            lines.append("vn %s %s %s" % tuple(repr(float(x)) for x in n[t, k].astype(np.float32)))
        b = 3 * t + 1
        lines.append(f"f {b}//{b} {b + 1}//{b + 1} {b + 2}//{b + 2}")
    p = tmp_path / "bunny.obj"
    p.write_text("\n".join(lines) + "\n")
    m = load_obj(p, None)
    s = scenes.main_scene((m.vertices, m.normals))
    orc = oracle.OracleScene(s.spec())
    tile = Tile(20, 52, 30, 54)
    got = render_samples(s, tile, 96, 128, 2, 0x5EED0001)
    want = orc.render_samples(tile, 96, 128, 2, 0x5EED0001, 0, oracle.MODE_REFERENCE, 8)
    assert np.array_equal(got["bounces"], want["bounces"])
    assert np.array_equal(got["flags"], want["flags"])
    assert np.array_equal(got["wavelength"], want["wavelength"])
    np.testing.assert_allclose(got["intensity"], want["intensity"], rtol=1e-12, atol=0)

"""The C-ABI library loads and exports every function include/vanrijn_amd.h declares (CPU only,
no compute calls that need a GPU)."""
import ctypes as C
import os
import re

import numpy as np

from vanrijn_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    text = open(os.path.join(ROOT, "include", "vanrijn_amd.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vr_[a-z0-9_]+)\s*\(", text)))


def test_every_declared_symbol_is_exported():
    lib = N.lib()
    names = declared_functions()
    assert len(names) >= 18
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(N.SIGNATURES) == names  # the Python binding covers exactly the header


def test_struct_sizes_match_header():
    assert C.sizeof(N.Spectrum) == 32
    assert C.sizeof(N.MaterialDesc) == 64
    assert C.sizeof(N.PrimitiveDesc) == 40
    assert C.sizeof(N.MeshDesc) == 32
    assert C.sizeof(N.ObjectDesc) == 16
    assert C.sizeof(N.SceneDesc) == 80
    assert C.sizeof(N.RenderParams) == 72
    assert C.sizeof(N.SampleRecord) == 48
    assert C.sizeof(N.HitRecord) == 144


def test_abi_version_and_error_strings():
    lib = N.lib()
    assert lib.vr_abi_version() == 3
    assert isinstance(lib.vr_last_error(), bytes)


def test_host_only_scene_and_errors():
    from vanrijn_amd import scenes
    from vanrijn_amd.render import Tile, render_tile
    s = scenes.bench_scene(scenes.displaced_mesh(6, [], 1, 0, 0.0, (1, 1, 1), (0, 0, 0)))
    ds = s.device_scene(0, host_only=True)
    info = ds.info()
    assert info["triangle_count"] == 12 * 36 and info["device_bytes"] == 0
    try:
        render_tile(ds, Tile(0, 2, 0, 2), 2, 2, 1, seed=1)
    except N.VrError as e:
        assert e.code == -8  # VR_ERROR_HOST_ONLY: no silent CPU path
    else:
        raise AssertionError("render on a host-only scene must fail")


def test_load_obj_fan_triangulation(tmp_path):
    p = tmp_path / "quad.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nvn 0 0 1\nf 1//1 2//1 3//1 4//1\nf -4 -2 -1\n")
    from vanrijn_amd.scene import load_obj
    m = load_obj(p, None)
    assert m.vertices.shape == (3, 3, 3)
    assert np.array_equal(m.vertices[0], [[0, 0, 0], [1, 0, 0], [1, 1, 0]])
    assert np.array_equal(m.vertices[1], [[0, 0, 0], [1, 1, 0], [0, 1, 0]])
    assert np.array_equal(m.normals[0], [[0, 0, 1]] * 3)
    assert np.array_equal(m.normals[2], np.zeros((3, 3)))  # no vn: zero normals (mesh.rs:31)
    # f32 parse then widen (mesh.rs:21-28)
    p.write_text("v 0.1 0.2 0.3\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    m = load_obj(p, None)
    assert m.vertices[0, 0, 0] == float(np.float32(0.1))


def test_load_obj_missing_file_is_io_error(tmp_path):
    from vanrijn_amd.scene import load_obj
    try:
        load_obj(tmp_path / "nope.obj", None)
    except N.VrError as e:
        assert e.code == -6
    else:
        raise AssertionError

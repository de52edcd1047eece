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
    assert C.sizeof(N.LaunchTimes) == 32
    assert C.sizeof(N.LaunchStats) == 96


def test_abi_version_and_error_strings():
    lib = N.lib()
    assert lib.vr_abi_version() == 10
    assert isinstance(lib.vr_last_error(), bytes)


def test_wide_offset_limits():
    """The default kernels address triangles (80-B TriVerts) and 4-wide nodes (128 B) with 32-bit
    byte offsets; past 4 GB of triangles or 2^25 wide nodes a scene takes the 64-bit-offset kernels
    (vr_render.hip render_kernel<.., BIG>; ADVICE r04: before, such a mesh silently read the wrong
    records).  Host only: the choice, at and either side of both limits."""
    f = N.lib().vr_scene_needs_wide_offsets
    tri_limit = (1 << 32) // 80 + 1  # the first count whose last record's offset reaches 2^32
    assert f(tri_limit - 1, 0) == 0 and f(tri_limit, 0) == 1
    assert f(53_687_091, 0) == 0 and f(53_687_092, 0) == 1
    assert f(1_051_392, 413_444) == 0  # C5's mesh and tree
    assert f(1000, (1 << 25) - 1) == 0 and f(1000, 1 << 25) == 1
    assert f((1 << 31) - 1, 1 << 30) == 1


def test_debug_launch_flags_validated():
    """vr_debug_set_launch_flags takes only the flags that leave records bit-identical."""
    from vanrijn_amd import scenes
    ds = scenes.bench_scene(scenes.displaced_mesh(6, [], 1, 0, 0.0, (1, 1, 1), (0, 0, 0))).device_scene(
        0, host_only=True)
    ds.set_launch_flags(no_cull=True, no_dist_cull=True, no_coop=True, no_lone_walk=True)
    ds.set_launch_flags()
    try:
        N.check(N.lib().vr_debug_set_launch_flags(ds.handle, N.LAUNCH_TIMED))
    except N.VrError as e:
        assert e.code == -1
    else:
        raise AssertionError("a timing flag is not a scene-wide debug flag")


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


def test_merge_tile_matches_oracle(oracle):
    """vr_merge_tile (host code in the library) == the oracle's merge_tile (accumulation_buffer.rs:62-85)."""
    from vanrijn_amd.render import AccumulationBuffer, Tile
    g = np.random.default_rng(5)
    W, H = 13, 9
    dst = AccumulationBuffer(W, H)
    dst.colour_buffer[...] = g.uniform(0, 2, (H, W, 3))
    dst.weight_buffer[...] = g.integers(1, 9, (H, W)).astype(float)
    t = Tile(3, 10, 2, 7)
    src = AccumulationBuffer(t.width(), t.height())
    src.colour_buffer[...] = g.uniform(0, 2, (t.height(), t.width(), 3))
    src.weight_buffer[...] = g.integers(1, 9, (t.height(), t.width())).astype(float)
    ref_c, ref_w = dst.colour_buffer.copy(), dst.weight_buffer.copy()
    oracle.lib().orc_merge_tile(W, ref_c.ctypes.data, ref_w.ctypes.data, t.start_row, t.start_column, t.height(),
                                t.width(), src.colour_buffer.ctypes.data, src.weight_buffer.ctypes.data)
    dst.merge_tile(t, src)
    assert np.array_equal(dst.colour_buffer, ref_c) and np.array_equal(dst.weight_buffer, ref_w)
    try:
        dst.merge_tile(Tile(0, 3, 0, 3), src)  # size mismatch: the reference asserts (accumulation_buffer.rs:63-64)
    except N.VrError as e:
        assert e.code == -1
    else:
        raise AssertionError("mismatched merge_tile must fail")


def test_merge_tile_large_tile_threaded(oracle):
    """A tile large enough to be split over host threads merges exactly like the oracle."""
    from vanrijn_amd.render import AccumulationBuffer, Tile
    g = np.random.default_rng(6)
    W, H = 700, 300
    dst = AccumulationBuffer(W, H)
    dst.colour_buffer[...] = g.uniform(0, 2, (H, W, 3))
    dst.weight_buffer[...] = g.integers(1, 9, (H, W)).astype(float)
    t = Tile(1, 699, 3, 297)
    src = AccumulationBuffer(t.width(), t.height())
    src.colour_buffer[...] = g.uniform(0, 2, (t.height(), t.width(), 3))
    src.weight_buffer[...] = g.integers(1, 9, (t.height(), t.width())).astype(float)
    ref_c, ref_w = dst.colour_buffer.copy(), dst.weight_buffer.copy()
    oracle.lib().orc_merge_tile(W, ref_c.ctypes.data, ref_w.ctypes.data, t.start_row, t.start_column, t.height(),
                                t.width(), src.colour_buffer.ctypes.data, src.weight_buffer.ctypes.data)
    for _ in range(3):  # the host pool is reused across calls
        d = AccumulationBuffer(W, H)
        d.colour_buffer[...] = dst.colour_buffer
        d.weight_buffer[...] = dst.weight_buffer
        d.merge_tile(t, src)
        assert np.array_equal(d.colour_buffer, ref_c) and np.array_equal(d.weight_buffer, ref_w)


def test_output_buffers_recycle_only_unreferenced_memory():
    """partial_render_scene's output buffers reuse memory of dropped buffers, never of live arrays."""
    import gc

    from vanrijn_amd.render import AccumulationBuffer
    a = AccumulationBuffer._for_output(40, 20)
    kept = a.weight_bias_buffer  # the caller keeps one array of an otherwise dropped buffer
    kept[...] = 7.0
    del a
    gc.collect()
    b = AccumulationBuffer._for_output(40, 20)
    for arr in (b.colour_buffer, b.colour_sum_buffer, b.colour_bias_buffer, b.weight_buffer, b.weight_bias_buffer):
        assert not np.shares_memory(arr, kept)
        arr[...] = -1.0
    assert (kept == 7.0).all()
    ptr = b.colour_buffer.ctypes.data
    del b, arr
    gc.collect()
    c = AccumulationBuffer._for_output(40, 20)  # b's store is free again
    assert c.colour_buffer.ctypes.data == ptr
    assert c.colour_buffer.shape == (20, 40, 3) and c.weight_buffer.shape == (20, 40)


def test_output_pool_respects_derived_views():
    """A slice or reshape of an output array (its numpy .base is the pooled store itself, not the
    view the pool handed out) keeps the store out of reuse after the buffer is dropped."""
    import gc

    from vanrijn_amd.render import AccumulationBuffer
    for derive in (lambda b: b.weight_bias_buffer[:, :], lambda b: b.colour_buffer[..., 0],
                   lambda b: b.colour_sum_buffer.reshape(-1), lambda b: b.weight_buffer[3:5, 1::2]):
        a = AccumulationBuffer._for_output(24, 12)
        kept = derive(a)
        kept[...] = 7.0
        del a
        gc.collect()
        b = AccumulationBuffer._for_output(24, 12)
        for arr in (b.colour_buffer, b.colour_sum_buffer, b.colour_bias_buffer, b.weight_buffer, b.weight_bias_buffer):
            assert not np.shares_memory(arr, kept)
            arr[...] = -1.0
        assert (kept == 7.0).all()
        del b, arr, kept
        gc.collect()

"""GPU parity: the gfx950 kernels (through the C ABI) against the oracle's reference mode.

Bar (DESIGN.md "Parity"):
  * decisions bit-identical: hit/miss, hit object/primitive, bounce counts, recursion-limit flags,
    wavelengths -- compared exactly;
  * closest-hit geometry (distance, location, normal, tangent, cotangent, retro) bit-identical;
  * per-sample intensities within 1e-12 relative (the kernel accumulates path throughput forward,
    the reference recursively: different association, same decisions);
  * per-pixel mean XYZ: L2 error < 1e-5 (north_star) -- observed ~1e-15.
At full size (1024^2, bench config) the checks are size-independent properties: tile and launch
split invariance (bitwise), continuation == single call (bitwise), finiteness, weights == spp.
"""
import numpy as np
import pytest

from vanrijn_amd import scenes
from vanrijn_amd.render import (AccumulationBuffer, Tile, partial_render_scene, render_samples, render_tile,
                                trace_rays)

pytestmark = pytest.mark.gpu

XYZ_L2_TOL = 1e-5          # north_star: per-pixel L2 error < 1e-5 vs reference
INTENSITY_REL_TOL = 1e-12  # forward vs recursive throughput association


@pytest.fixture(scope="module")
def bunny():
    return scenes.procedural_bunny()


@pytest.fixture(scope="module")
def main_pair(bunny, oracle):
    s = scenes.main_scene(bunny)
    return s, oracle.OracleScene(s.spec())


@pytest.fixture(scope="module")
def bench_pair(bunny, oracle):
    s = scenes.bench_scene(bunny)
    return s, oracle.OracleScene(s.spec())


def _compare_hits(gpu, ref):
    assert len(gpu) == len(ref)
    valid = np.array([h.valid for h in ref], dtype=bool)
    assert np.array_equal(gpu["valid"].astype(bool), valid)
    obj = np.array([h.object for h in ref])[valid]
    prim = np.array([h.primitive for h in ref])[valid]
    assert np.array_equal(gpu["object"][valid], obj)
    assert np.array_equal(gpu["primitive"][valid], prim)
    dist = np.array([h.distance for h in ref])[valid]
    assert np.array_equal(gpu["distance"][valid], dist)
    for f in ("location", "normal", "tangent", "cotangent", "retro"):
        r = np.array([list(getattr(h, f)) for h in ref])[valid]
        g = gpu[f][valid]
        same = (g == r) | (np.isnan(g) & np.isnan(r))
        assert same.all(), f


def _ray_batch(spec, n, seed):
    g = np.random.default_rng(seed)
    cam = np.array(spec.camera_location)
    tgt = g.uniform([-3.5, -2.5, -1.5], [0.5, 1.5, 1.5], (n, 3))
    o = np.concatenate([np.repeat(cam[None], n, 0), g.uniform([-3.5, -1.9, -1.5], [0.0, 1.2, 1.3], (n, 3))])
    d = np.concatenate([tgt - cam, g.normal(size=(n, 3))])
    d = d / np.linalg.norm(d, axis=1, keepdims=True)
    return o, d


def test_trace_rays_bitwise(main_pair, oracle):
    scene, orc = main_pair
    o, d = _ray_batch(scene.spec(), 4000, 1)
    ref, _ = orc.trace(o, d, oracle.MODE_REFERENCE)
    _compare_hits(trace_rays(scene, o, d), ref)


def test_trace_rays_from_surface_points(main_pair, oracle):
    """Bounce-like rays: origins on the mesh (hit points + 1e-7 bias), random directions."""
    scene, orc = main_pair
    o, d = _ray_batch(scene.spec(), 3000, 2)
    first, _ = orc.trace(o[:3000], d[:3000], oracle.MODE_REFERENCE)
    pts = np.array([list(h.location) for h in first if h.valid])
    g = np.random.default_rng(3)
    dirs = g.normal(size=pts.shape)
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    origins = pts + dirs * 1e-7
    ref, _ = orc.trace(origins, dirs, oracle.MODE_REFERENCE)
    _compare_hits(trace_rays(scene, origins, dirs), ref)


@pytest.mark.parametrize("which", ["main", "bench"])
def test_samples_decision_identical(which, main_pair, bench_pair, oracle):
    scene, orc = main_pair if which == "main" else bench_pair
    H = W = 96
    t = Tile(24, 72, 30, 78)
    ref = orc.render_samples(t, H, W, 4, seed=0x5EED0001, mode=oracle.MODE_REFERENCE, nthreads=8)
    gpu = render_samples(scene, t, H, W, 4, seed=0x5EED0001)
    assert np.array_equal(gpu["flags"], ref["flags"])
    assert np.array_equal(gpu["bounces"], ref["bounces"])
    assert np.array_equal(gpu["wavelength"], ref["wavelength"])
    den = np.maximum(np.abs(ref["intensity"]), 1e-300)
    rel = np.abs(gpu["intensity"] - ref["intensity"]) / den
    assert (rel[ref["intensity"] != 0] < INTENSITY_REL_TOL).all()
    assert np.array_equal(gpu["intensity"] == 0, ref["intensity"] == 0)
    assert (ref["flags"] & 1).sum() > 100


@pytest.mark.parametrize("which", ["main", "bench"])
def test_image_parity_l2(which, main_pair, bench_pair, oracle):
    scene, orc = main_pair if which == "main" else bench_pair
    H, W = 64, 80  # non-square: film (w/h, 1)
    t = Tile(0, W, 0, H)
    ref = orc.render_tile(t, H, W, 16, seed=7, mode=oracle.MODE_REFERENCE, nthreads=8)
    gpu = render_tile(scene, t, H, W, 16, seed=7)
    err = np.linalg.norm(gpu.colour_buffer - ref["colour"], axis=2)
    assert err.max() < XYZ_L2_TOL
    assert np.array_equal(gpu.weight_buffer, ref["weight"])


def test_partial_render_scene_contract(main_pair):
    scene, _ = main_pair
    t = Tile(3, 19, 5, 13)
    a = partial_render_scene(scene, t, 32, 24)
    b = partial_render_scene(scene, t, 32, 24)
    assert a.width() == 16 and a.height() == 8
    assert np.array_equal(a.weight_buffer, np.ones((8, 16)))
    assert np.isfinite(a.colour_buffer).all()
    # successive calls draw different sample indices (fresh randomness like thread_rng)
    assert not np.array_equal(a.colour_buffer, b.colour_buffer)
    # merge_tile of the two passes == their blend
    full = AccumulationBuffer(24, 32)
    full.merge_tile(t, a)
    full.merge_tile(t, b)
    assert np.allclose(full.colour_buffer[5:13, 3:19], (a.colour_buffer + b.colour_buffer) / 2, rtol=0, atol=1e-15)


def test_one_sample_fresh_buffer_fast_path(main_pair):
    """vr_render_tile with spp 1 into a fresh buffer brings back only colour_sum and derives the other
    four arrays on the host; it equals update_pixel on an explicit all-zero buffer (the general
    path: all five arrays through the device) bit for bit."""
    scene, _ = main_pair
    H, W = 300, 260  # > 64k pixels: the host expansion runs on several threads
    t = Tile(0, W, 0, H)
    fast = render_tile(scene, t, H, W, 1, seed=11, first_sample=5)
    general = render_tile(scene, t, H, W, 1, seed=11, first_sample=5, accumulate=AccumulationBuffer(W, H))
    for k in ("colour_sum_buffer", "colour_bias_buffer", "weight_buffer", "weight_bias_buffer", "colour_buffer"):
        assert np.array_equal(getattr(fast, k), getattr(general, k), equal_nan=True), k
    assert np.array_equal(fast.weight_buffer, np.ones((H, W)))


def test_staging_pass_split_is_one_launch(main_pair):
    """A frame whose staging exceeds the per-launch cap runs in passes that continue update_pixel in
    sample order: the records equal one launch bit for bit (vr_scene_set_staging_limit forces 16
    passes)."""
    import torch
    from vanrijn_amd.render import _scene_handle, render_tile_device
    scene, _ = main_pair
    ds = _scene_handle(scene, 0)
    H, W, spp = 256, 256, 16
    t = Tile(0, W, 0, H)
    one = torch.zeros(H * W * 8, dtype=torch.float64, device="cuda")
    st1 = render_tile_device(ds, t, H, W, spp, 9, 0, one.data_ptr(), timed=True)
    split = torch.zeros_like(one)
    ds.set_staging_limit(1 << 20)  # 1 MiB = one sample of 65536 pixels per pass
    try:
        st2 = render_tile_device(ds, t, H, W, spp, 9, 0, split.data_ptr(), timed=True)
    finally:
        ds.set_staging_limit(0)
    assert st1["passes"] == 1 and st2["passes"] == spp
    assert torch.equal(one, split)


def test_tile_invariance_and_continuation(main_pair):
    scene, _ = main_pair
    H, W = 48, 40
    full = render_tile(scene, Tile(0, W, 0, H), H, W, 6, seed=3)
    for t in (Tile(0, 17, 0, 9), Tile(17, 40, 9, 48), Tile(5, 6, 30, 31)):
        part = render_tile(scene, t, H, W, 6, seed=3)
        assert np.array_equal(part.colour_sum_buffer, full.colour_sum_buffer[t.start_row:t.end_row,
                                                                             t.start_column:t.end_column])
    split = render_tile(scene, Tile(0, W, 0, H), H, W, 2, seed=3)
    split = render_tile(scene, Tile(0, W, 0, H), H, W, 4, seed=3, first_sample=2, accumulate=split)
    for k in ("colour_sum_buffer", "colour_bias_buffer", "weight_buffer", "weight_bias_buffer", "colour_buffer"):
        assert np.array_equal(getattr(split, k), getattr(full, k)), k


def test_edge_cases(bunny, oracle):
    from vanrijn_amd.scene import (BoundingVolumeHierarchy, LambertianMaterial, Mesh, Scene, Spectrum)
    mat = LambertianMaterial(Spectrum.grey(0.8), 0.5)
    # empty mesh, single triangle, 1x1 image, portrait image
    empty = Scene((0, 0, -3), [BoundingVolumeHierarchy.build(Mesh(np.zeros((0, 3, 3)), np.zeros((0, 3, 3)), mat))])
    b = render_tile(empty, Tile(0, 4, 0, 4), 4, 4, 2, seed=1)
    assert np.array_equal(b.colour_buffer, np.zeros((4, 4, 3))) and np.array_equal(b.weight_buffer, np.full((4, 4), 2.0))
    tri = np.array([[[-1, -1, 0], [1, -1, 0], [0, 1, 0]]], float)
    one = Scene((0, 0, -3), [BoundingVolumeHierarchy.build(Mesh(tri, np.tile([0, 0, -1.0], (1, 3, 1)), mat))])
    orc = oracle.OracleScene(one.spec())
    for (h, w) in ((1, 1), (8, 3), (3, 8)):
        t = Tile(0, w, 0, h)
        ref = orc.render_samples(t, h, w, 8, seed=5, mode=oracle.MODE_REFERENCE)
        gpu = render_samples(one, t, h, w, 8, seed=5)
        assert np.array_equal(gpu["flags"], ref["flags"]) and np.array_equal(gpu["bounces"], ref["bounces"])
    # empty tile is a no-op
    z = render_tile(one, Tile(2, 2, 1, 1), 4, 4, 3, seed=1)
    assert z.colour_buffer.size == 0


def test_invalid_tile_is_an_error(main_pair):
    from vanrijn_amd._native import VrError
    scene, _ = main_pair
    with pytest.raises(VrError):
        render_tile(scene, Tile(0, 10, 0, 10), 8, 8, 1, seed=1)


def test_random_stream_index_space_is_enforced(main_pair):
    """The stream base mix64(key ^ (pixel << 32 | sample)) is injective only below 2^32 pixels and
    samples: sample ranges past 2^32 and images of more than 2^32
    pixels are refused, the last representable sample renders."""
    from vanrijn_amd._native import VrError
    scene, _ = main_pair
    t = Tile(0, 4, 0, 4)
    with pytest.raises(VrError) as e:
        render_tile(scene, t, 8, 8, 2, seed=1, first_sample=(1 << 32) - 1)
    assert e.value.code == -7  # VR_ERROR_UNSUPPORTED
    with pytest.raises(VrError):
        render_tile(scene, t, 1 << 17, 1 << 16, 1, seed=1)
    ok = render_tile(scene, t, 8, 8, 1, seed=1, first_sample=(1 << 32) - 1)
    assert np.array_equal(ok.weight_buffer, np.ones((4, 4)))


def test_full_size_properties(bench_pair):
    """Bench config size (1024^2) at low spp: invariances that hold at any size."""
    scene, _ = bench_pair
    H = W = 1024
    a = render_tile(scene, Tile(0, W, 0, H), H, W, 2, seed=0x5EED0001)
    assert np.isfinite(a.colour_buffer).all()
    assert np.array_equal(a.weight_buffer, np.full((H, W), 2.0))
    b = render_tile(scene, Tile(256, 768, 512, 1024), H, W, 2, seed=0x5EED0001)
    assert np.array_equal(b.colour_sum_buffer, a.colour_sum_buffer[512:1024, 256:768])

"""Launch variants that must not change a bit of the records, through the C ABI on the GPU.

* VR_LAUNCH_NO_DIST_CULL: the BVH distance culling off, so every box the ray's line crosses is walked
  as in the reference's exhaustive traversal (bounding_volume_hierarchy.rs:94-120).  Round 4 found a
  tie rule miscompiled in a way the culling order had hidden ("A miscompiled tie
  rule"): the tie scenes (test_gpu_ties.py) and the tie / flat meshes of test_gpu_build.py are decided
  here with the culling off, against the oracle's reference mode -- the later in-order leaf wins inside
  a BVH (bvh.rs:77-92), the earlier object across objects (sampler.rs:9-20).
* VR_LAUNCH_NO_COOP: the cooperative tail (vr_render.hip coop_step, the COOP instantiations small
  launches of mirror scenes take) against the plain kernel, bit for bit, on the C1 scene
  (benches/simple_scene.rs), whose paths trapped between mirror facets run to the 128-bounce limit.
* VR_SCENE_WIDE_OFFSETS: the 64-bit-offset kernels that scenes past 4 GB of triangles or 2^25 wide
  nodes take, forced on small scenes, against the default kernels bit for bit.
"""
import numpy as np
import pytest
import torch

from vanrijn_amd import _native as N
from vanrijn_amd import scenes
from vanrijn_amd.render import Tile, render_samples, render_tile, render_tile_device
from vanrijn_amd.scene import DeviceScene

from test_gpu_build import _mesh_scene, _random_mesh
from test_gpu_ties import INTENSITY_REL_TOL, _tied_scene

pytestmark = pytest.mark.gpu


def _decisions_equal(gpu, ref):
    assert np.array_equal(gpu["flags"], ref["flags"])
    assert np.array_equal(gpu["bounces"], ref["bounces"])
    assert np.array_equal(gpu["wavelength"], ref["wavelength"])
    den = np.maximum(np.abs(ref["intensity"]), 1e-300)
    rel = np.abs(gpu["intensity"] - ref["intensity"]) / den
    ok = (ref["intensity"] == 0) | (rel < INTENSITY_REL_TOL) | (np.isnan(ref["intensity"]) & np.isnan(gpu["intensity"]))
    assert ok.all()


@pytest.mark.parametrize("seed", [1, 2])
def test_ties_without_distance_culling(seed, oracle):
    scene = _tied_scene(seed)
    ds = DeviceScene(scene.spec(), 0)
    ds.set_launch_flags(no_dist_cull=True)
    orc = oracle.OracleScene(scene.spec())
    H = W = 64
    t = Tile(0, W, 0, H)
    ref = orc.render_samples(t, H, W, 6, seed=0x7135 + seed, mode=oracle.MODE_REFERENCE, nthreads=8)
    gpu = render_samples(ds, t, H, W, 6, seed=0x7135 + seed)
    assert (ref["flags"] & 1).sum() > 1000
    _decisions_equal(gpu, ref)
    # the timed instantiation (early stop, frustum culling, ordered reduce) without distance culling
    img = render_tile(ds, t, H, W, 6, seed=0x7135 + seed)
    refi = orc.render_tile(t, H, W, 6, seed=0x7135 + seed, mode=oracle.MODE_PRUNED, nthreads=8)
    assert np.linalg.norm(img.colour_buffer - refi["colour"], axis=2).max() < 1e-5
    assert np.array_equal(img.weight_buffer, refi["weight"])
    # and the device records equal the culled render's bit for bit
    on = DeviceScene(scene.spec(), 0)
    a = torch.zeros(H * W * 8, dtype=torch.float64, device="cuda")
    b = torch.zeros_like(a)
    render_tile_device(on, t, H, W, 6, 0x7135 + seed, 0, a.data_ptr())
    render_tile_device(on, t, H, W, 6, 0x7135 + seed, 0, b.data_ptr(), dist_cull=False)
    torch.cuda.synchronize()
    assert torch.equal(a.view(torch.int64), b.view(torch.int64))


@pytest.mark.parametrize("kind", ["ties", "flat"])
def test_build_meshes_without_distance_culling(kind, oracle):
    """test_gpu_build.py's degenerate meshes (centroids on a half-integer grid: coplanar triangles tie
    at equal distances; one axis without extent), reference and SAH trees, decided with the culling
    off like the oracle's reference mode."""
    rng = np.random.default_rng(11)
    scene = _mesh_scene(_random_mesh(rng, 3000, ties=kind == "ties", flat=kind == "flat"))
    orc = oracle.OracleScene(scene.spec())
    H, W = 40, 48
    t = Tile(0, W, 0, H)
    ref = orc.render_samples(t, H, W, 3, seed=0x5EED0001, mode=oracle.MODE_REFERENCE, nthreads=8)
    assert (ref["flags"] & 1).sum() > 500
    for kw in ({}, {"reference_bvh": True}, {"device_sah": True}):
        ds = DeviceScene(scene.spec(), 0, **kw)
        ds.set_launch_flags(no_dist_cull=True)
        _decisions_equal(render_samples(ds, t, H, W, 3, seed=0x5EED0001), ref)


def test_cooperative_tail_is_bit_identical():
    """C1 (benches/simple_scene.rs: reflective bunny, 256^2 @16): the COOP instantiation runs (the
    launch reports it) and its records equal the plain kernel's, fresh and accumulating -- with the
    whole-walk form (lone_walk, one and two owners per wave) and in coop_step's per-step form only."""
    ds = scenes.bench_scene().device_scene(0)
    H = W = 256
    t = Tile(0, W, 0, H)
    stream = torch.cuda.current_stream().cuda_stream
    out = []
    for coop, lone in ((True, True), (True, False), (False, True)):
        st = torch.zeros(H * W * 8, dtype=torch.float64, device="cuda")
        s1 = render_tile_device(ds, t, H, W, 16, 0x5EED0001, 0, st.data_ptr(), stream, coop=coop, lone_walk=lone)
        s2 = render_tile_device(ds, t, H, W, 5, 0x5EED0001, 16, st.data_ptr(), stream, accumulate=True, coop=coop,
                                lone_walk=lone)
        torch.cuda.synchronize()
        assert bool(s1["variant"] & N.VARIANT_COOP) == coop and bool(s2["variant"] & N.VARIANT_COOP) == coop
        out.append(st.cpu())
    for o in out[1:]:
        assert torch.equal(out[0].view(torch.int64), o.view(torch.int64))
    assert np.isfinite(out[0].numpy()).all()


def test_cooperative_tail_matches_the_oracle_on_a_crop(oracle):
    """The COOP launch's image against the oracle on a crop where mirror paths run long."""
    scene = scenes.bench_scene()
    ds = scene.device_scene(0)
    t = Tile(96, 160, 96, 160)
    img = render_tile(ds, t, 256, 256, 16, seed=0x5EED0001)
    refi = oracle.OracleScene(scene.spec()).render_tile(t, 256, 256, 16, seed=0x5EED0001, mode=oracle.MODE_PRUNED,
                                                        nthreads=8)
    assert np.linalg.norm(img.colour_buffer - refi["colour"], axis=2).max() < 1e-5
    assert np.array_equal(img.weight_buffer, refi["weight"])


def _two_mirror_scene():
    """Two reflective bunny-like meshes side by side (two mesh BVHs; the second one's root is not node
    0), close enough that paths bounce between them: the cooperative tail's owners then walk either
    BVH from lanes other than 0 / 32 (a walk that starts at the wrong node, or at the
    first BVH's root, is invisible on bench_scene's single mesh)."""
    from vanrijn_amd.scene import (BoundingVolumeHierarchy, ColourRgbF, Mesh, NamedColour, ReflectiveMaterial, Scene,
                                   Spectrum)
    objs = []
    for centre, seed, colour in (((-2.55, -0.5, 0.0), 0xB0BB1E, NamedColour.Yellow),
                                 ((-0.95, -0.35, 0.25), 0xC0FFEE, NamedColour.Red)):
        v, n = scenes.displaced_mesh(20, scenes._BUNNY_BUMPS, noise_seed=seed, noise_count=24, noise_amp=0.05,
                                     scale=(0.8, 0.75, 0.8), centre=centre)
        mat = ReflectiveMaterial(Spectrum.reflection_from_linear_rgb(ColourRgbF.from_named(colour)), 0.05, 0.9)
        objs.append(BoundingVolumeHierarchy.build(Mesh(v, n, mat)))
    return Scene(scenes.CAMERA_LOCATION, objs)


def test_cooperative_tail_two_mirror_meshes(oracle):
    """The cooperative tail on a scene of two mirror meshes: whole walks (lone_walk), per-step walks
    (coop_step) and the plain kernel give the same records bit for bit, fresh and accumulating, the
    COOP kernel is the one reported, and a crop where paths run long matches the oracle."""
    scene = _two_mirror_scene()
    ds = scene.device_scene(0)
    H = W = 160
    t = Tile(0, W, 0, H)
    stream = torch.cuda.current_stream().cuda_stream
    out = []
    for coop, lone in ((True, True), (True, False), (False, True)):
        st = torch.zeros(H * W * 8, dtype=torch.float64, device="cuda")
        s1 = render_tile_device(ds, t, H, W, 16, 0x5EED0001, 0, st.data_ptr(), stream, coop=coop, lone_walk=lone)
        s2 = render_tile_device(ds, t, H, W, 5, 0x5EED0001, 16, st.data_ptr(), stream, accumulate=True, coop=coop,
                                lone_walk=lone)
        torch.cuda.synchronize()
        assert bool(s1["variant"] & N.VARIANT_COOP) == coop and bool(s2["variant"] & N.VARIANT_COOP) == coop
        out.append(st.cpu())
    for o in out[1:]:
        assert torch.equal(out[0].view(torch.int64), o.view(torch.int64))
    assert np.isfinite(out[0].numpy()).all()
    # against the oracle where the two meshes face each other, per sample (decisions) and as an image
    orc = oracle.OracleScene(scene.spec())
    crop = Tile(56, 104, 72, 120)
    ref = orc.render_samples(crop, H, W, 4, seed=0x5EED0001, mode=oracle.MODE_PRUNED, nthreads=8)
    assert (ref["bounces"] >= 8).sum() > 0  # some paths bounce between the mirrors
    img = render_tile(ds, crop, H, W, 16, seed=0x5EED0001)
    refi = orc.render_tile(crop, H, W, 16, seed=0x5EED0001, mode=oracle.MODE_PRUNED, nthreads=8)
    assert np.linalg.norm(img.colour_buffer - refi["colour"], axis=2).max() < 1e-5
    assert np.array_equal(img.weight_buffer, refi["weight"])
    _decisions_equal(render_samples(ds, crop, H, W, 4, seed=0x5EED0001), ref)


@pytest.mark.parametrize("which", ["main", "bench", "whitted", "materials"])
def test_wide_offset_kernels_are_bit_identical(which):
    """The 64-bit-offset kernels (forced) render the same records as the default ones, and the launch
    reports which ran."""
    scene = {"main": scenes.main_scene, "bench": scenes.bench_scene, "whitted": scenes.whitted_scene,
             "materials": scenes.materials_scene}[which]()
    H, W = 120, 160
    t = Tile(20, 140, 10, 110)
    npix = t.width() * t.height()
    out = []
    for wide in (False, True):
        ds = DeviceScene(scene.spec(), 0, device_sah=True, wide_offsets=wide)
        st = torch.zeros(npix * 8, dtype=torch.float64, device="cuda")
        s = render_tile_device(ds, t, H, W, 6, 0x5EED0001, 0, st.data_ptr())
        c = render_tile_device(ds, t, H, W, 2, 0x5EED0001, 6, st.data_ptr(), accumulate=True, counters=True)
        torch.cuda.synchronize()
        assert bool(s["variant"] & N.VARIANT_WIDE_OFFSETS) == wide
        assert bool(c["variant"] & N.VARIANT_WIDE_OFFSETS) == wide
        rec = render_samples(ds, t, H, W, 2, seed=0x5EED0001)
        out.append((st.cpu(), rec, c["node_visits"]))
    assert torch.equal(out[0][0].view(torch.int64), out[1][0].view(torch.int64))  # bitwise, NaN included
    assert out[0][1].tobytes() == out[1][1].tobytes()


@pytest.mark.parametrize("which", ["main", "bench_nocoop"])
def test_stack16_kernels_are_bit_identical(which):
    """16-bit traversal-stack entries (trees below 65,536 wide nodes: the bunny's 27 K) against the
    32-bit ones (VR_LAUNCH_STACK32), fresh and accumulating; the launch reports which ran."""
    scene = scenes.main_scene() if which == "main" else scenes.bench_scene()
    ds = scene.device_scene(0, device_sah=True)
    H, W = 200, 240
    t = Tile(16, 216, 20, 180)
    npix = t.width() * t.height()
    out = []
    for s16 in (True, False):
        st = torch.zeros(npix * 8, dtype=torch.float64, device="cuda")
        # the bench scene's small launches take the cooperative tail (32-bit stacks): without it
        a = render_tile_device(ds, t, H, W, 12, 0x5EED0001, 0, st.data_ptr(), coop=False, stack16=s16)
        b = render_tile_device(ds, t, H, W, 5, 0x5EED0001, 12, st.data_ptr(), accumulate=True, coop=False,
                               stack16=s16)
        torch.cuda.synchronize()
        assert bool(a["variant"] & N.VARIANT_STACK16) == s16 and bool(b["variant"] & N.VARIANT_STACK16) == s16
        out.append(st.cpu())
    assert torch.equal(out[0].view(torch.int64), out[1].view(torch.int64))


def test_stack16_needs_a_small_tree():
    """C5's 1.05 M-triangle mesh has ~413 K wide nodes: its kernels keep 32-bit stack entries."""
    ds = scenes.synthetic_scene().device_scene(0, device_sah=True)
    st = torch.zeros(64 * 64 * 8, dtype=torch.float64, device="cuda")
    s = render_tile_device(ds, Tile(0, 64, 0, 64), 64, 64, 1, 0x5EED0001, 0, st.data_ptr())
    torch.cuda.synchronize()
    assert not s["variant"] & N.VARIANT_STACK16

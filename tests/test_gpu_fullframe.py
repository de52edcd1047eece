"""Full-size parity of the timed kernel, image mode, against the oracle (camera.rs:95-130).

The timed launches run `render_kernel<.., RECORD = false, DARK0, MATS = 1>`: the instantiation
with the early stop of zero-throughput paths, camera-frustum culling of 8x8 blocks and the
dark-wave skip of the ordered reduce.  The decision tests (test_gpu_parity*.py) use the record
instantiation, which has none of these, so here the product's own image path is compared with the
oracle on whole BASELINE frames:

  * C3: the main.rs scene's full 1024x1024 frame at 16 spp (16.8 M samples);
  * C4: its full 2048x2048 frame at 4 spp (the frame's last samples, 1020..1023);
  * C5: the 1,051,392-triangle scene's full 4096x4096 frame at 1 spp (16.8 M samples);
  * a scene where the reference produces NaN: main.rs's scene plus a mesh loaded from an OBJ
    without normals (mesh.rs:37 gives it zero normals, so every hit on it has a NaN shading basis,
    triangle.rs:73-78).  The mesh stands behind the camera, where no camera ray reaches it, so every
    NaN sample first hit a normal'd object -- and those with a wavelength in (720, 740) nm, where
    every spectrum is 0, have zero throughput after that first hit: exactly the paths an early stop
    would end with intensity 0 while the reference returns inner x 0 = NaN
    (simple_random_integrator.rs:39-53).

Bar: weights exact, NaN pixels identical (equal_nan), per-pixel mean XYZ L2 < 1e-5 elsewhere
(north_star).  C3 and C5 use the oracle's pruned mode (the reference-mode closest hit, distance-
culled: tests/test_oracle_scene.py checks the two equal, on C5's mesh too); the NaN scene uses
reference mode.
"""
import os

import numpy as np
import pytest

from vanrijn_amd import scenes
from vanrijn_amd.render import Tile, render_samples, render_tile
from vanrijn_amd.scene import BoundingVolumeHierarchy, LambertianMaterial, Scene, Spectrum, load_obj
from vanrijn_amd.scene import ColourRgbF

pytestmark = pytest.mark.gpu

XYZ_L2_TOL = 1e-5
SEED = 0x5EED0001
THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


def _compare_images(gpu, ref, spp, shape):
    g, r = gpu.colour_buffer, ref["colour"]
    assert np.array_equal(gpu.weight_buffer, ref["weight"])
    assert np.array_equal(gpu.weight_buffer, np.full(shape, float(spp)))
    gnan, rnan = np.isnan(g).any(axis=2), np.isnan(r).any(axis=2)
    assert np.array_equal(gnan, rnan), (int(gnan.sum()), int(rnan.sum()))
    ok = ~rnan
    err = np.linalg.norm(g[ok] - r[ok], axis=1)
    assert err.max() < XYZ_L2_TOL, float(err.max())
    return int(rnan.sum()), float(err.max())


def test_c3_full_frame_16spp(oracle):
    s = scenes.main_scene()
    ds = s.device_scene(0)
    assert ds.info()["nan_free"]  # the headline scene keeps the early stop
    t = Tile(0, 1024, 0, 1024)
    gpu = render_tile(ds, t, 1024, 1024, 16, seed=SEED)
    ref = oracle.OracleScene(s.spec()).render_tile(t, 1024, 1024, 16, seed=SEED, mode=oracle.MODE_PRUNED,
                                                   nthreads=THREADS)
    nans, err = _compare_images(gpu, ref, 16, (1024, 1024))
    assert nans == 0
    print(f"C3 full frame @16 spp: max per-pixel XYZ L2 error {err:.3e}")


def test_c4_full_frame_4spp(oracle):
    """C4's frame size (BASELINE configs[3]: 2048x2048, the main.rs scene) in full at 4 spp (16.8 M
    samples) -- until round 6 only a 64x64 crop of it was checked."""
    s = scenes.main_scene()
    ds = s.device_scene(0)
    t = Tile(0, 2048, 0, 2048)
    gpu = render_tile(ds, t, 2048, 2048, 4, seed=SEED, first_sample=1020)
    ref = oracle.OracleScene(s.spec()).render_tile(t, 2048, 2048, 4, seed=SEED, first_sample=1020,
                                                   mode=oracle.MODE_PRUNED, nthreads=THREADS)
    nans, err = _compare_images(gpu, ref, 4, (2048, 2048))
    assert nans == 0
    print(f"C4 full frame @4 spp (samples 1020..1023): max per-pixel XYZ L2 error {err:.3e}")


def test_c5_full_frame_1spp(oracle):
    s = scenes.synthetic_scene()
    ds = s.device_scene(0)
    assert ds.info()["triangle_count"] == 1_051_392 and ds.info()["nan_free"]
    t = Tile(0, 4096, 0, 4096)
    gpu = render_tile(ds, t, 4096, 4096, 1, seed=SEED)
    ref = oracle.OracleScene(s.spec()).render_tile(t, 4096, 4096, 1, seed=SEED, mode=oracle.MODE_PRUNED,
                                                   nthreads=THREADS)
    nans, err = _compare_images(gpu, ref, 1, (4096, 4096))
    assert nans == 0
    print(f"C5 full frame @1 spp: max per-pixel XYZ L2 error {err:.3e}")


def nan_scene(tmp_path):
    """main.rs's plane and spheres, a small Lambertian bunny, and a normal-less OBJ wall behind the
    camera (z = -7; the camera at z = -5 looks down +z)."""
    obj = tmp_path / "wall_without_normals.obj"
    obj.write_text("v -24 -2 -7\nv 16 -2 -7\nv 16 16 -7\nv -24 16 -7\nf 1 2 3 4\n")
    grey = LambertianMaterial(Spectrum.reflection_from_linear_rgb(ColourRgbF.new(0.5, 0.5, 0.5)), 0.1)
    wall = load_obj(obj, grey)
    assert len(wall.vertices) == 2 and not wall.normals.any()  # mesh.rs:37: zero normals
    small = scenes.displaced_mesh(8, scenes._BUNNY_BUMPS, 0xB0BB1E, 8, 0.04, (1.25, 1.05, 1.15), (-1.7, -0.8, 0.0))
    base = scenes.main_scene(small)
    return Scene(base.camera_location, base.objects + [BoundingVolumeHierarchy.build(wall)])


def test_normalless_mesh_nan_pixels_like_the_reference(oracle, tmp_path):
    s = nan_scene(tmp_path)
    ds = s.device_scene(0)
    assert not ds.info()["nan_free"]  # the zero normals: no early stop, the general lambda-0 chain
    assert scenes.main_scene().device_scene(0).info()["nan_free"]
    orc = oracle.OracleScene(s.spec())
    H, W, spp = 48, 48, 4
    t = Tile(0, W, 0, H)
    # samples: the reference's NaN photons include early-stop cases (camera ray on a normal'd
    # object, wavelength where every spectrum is 0, a later bounce into the wall)
    rec = orc.render_samples(t, H, W, spp, seed=SEED, mode=oracle.MODE_REFERENCE, nthreads=THREADS)
    gs = render_samples(ds, t, H, W, spp, seed=SEED)
    assert np.array_equal(np.isnan(gs["intensity"]), np.isnan(rec["intensity"]))
    assert np.array_equal(gs["flags"], rec["flags"]) and np.array_equal(gs["bounces"], rec["bounces"])
    assert np.array_equal(gs["wavelength"], rec["wavelength"])
    nan = np.isnan(rec["intensity"])
    assert nan.sum() > 100, int(nan.sum())
    # wavelength 0 after the recursion limit: the drawn wavelength is not in the record, so count
    # NaN samples whose path saw a dark first hit via the first bounce's draw -- at least the
    # camera-hit NaN samples exist and none started on the wall (behind the camera)
    assert ((rec["flags"] & 1)[nan] == 1).all()
    # image mode: the timed instantiation's path
    gpu = render_tile(ds, t, H, W, spp, seed=SEED)
    ref = orc.render_tile(t, H, W, spp, seed=SEED, mode=oracle.MODE_REFERENCE, nthreads=THREADS)
    nans, err = _compare_images(gpu, ref, spp, (H, W))
    assert nans > 50, nans
    print(f"NaN scene: {int(nan.sum())} NaN samples, {nans} NaN pixels, max finite-pixel L2 error {err:.3e}")


def test_dark_wavelength_paths_are_traced_not_stopped(oracle, tmp_path):
    """The early-stop case itself: per sample, the wavelength is the stream's third draw
    (0-based draw 2, camera.rs:114-118); samples with a wavelength in (720, 740) nm whose
    camera ray hits have zero throughput after their first hit, and those that later meet the wall
    are NaN in the reference.  The GPU's image must carry them as NaN (an early stop gives 0)."""
    s = nan_scene(tmp_path)
    ds = s.device_scene(0)
    orc = oracle.OracleScene(s.spec())
    H, W, spp = 48, 48, 4
    t = Tile(0, W, 0, H)
    rec = orc.render_samples(t, H, W, spp, seed=SEED, mode=oracle.MODE_REFERENCE, nthreads=THREADS)
    # the drawn wavelength of every sample from the counter-based stream (draw 3)
    rows, cols, ss = np.meshgrid(np.arange(H), np.arange(W), np.arange(spp), indexing="ij")
    lam = np.empty(rows.shape)
    for idx in np.ndindex(rows.shape):
        base = oracle.lib().orc_stream_base(SEED, int(rows[idx]) * W + int(cols[idx]), int(ss[idx]))
        lam[idx] = 380.0 + 360.0 * oracle.lib().orc_u64_to_standard(oracle.lib().orc_stream_draw(base, 2))
    dark = ((rec["flags"] & 1) == 1) & (lam > 720.0)
    dark_nan = dark & np.isnan(rec["intensity"])
    assert dark_nan.sum() >= 3, (int(dark.sum()), int(dark_nan.sum()))
    # their pixels are NaN in the GPU image (the reference's 0 * NaN), not finite
    gpu = render_tile(ds, t, H, W, spp, seed=SEED)
    pix = dark_nan.any(axis=2)
    assert np.isnan(gpu.colour_buffer[pix]).all()

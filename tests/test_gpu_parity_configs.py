"""GPU parity at the BASELINE.json configs' sizes, against the oracle.

  C1  bench scene (benches/simple_scene.rs:19-45), full 256x256 frame @16 spp
  C2  main.rs scene (src/main.rs:138-189), full 512x512 frame @64 spp
  C3  main.rs scene, a 128x128 crop of the 1024x1024 frame (global H = W = 1024) @32 spp
  C4  main.rs scene, a 64x64 crop of the 2048x2048 frame @16 spp
  C5  the 1,051,392-triangle synthetic mesh scene, a 64x64 crop of the 4096x4096 frame @4 spp

Every case checks, through the C ABI against the oracle:
  * per-sample decisions bit-identical (camera hit / recursion limit / singular flags, bounce
    counts, wavelengths) for every (pixel, sample) of the frame or crop;
  * per-sample intensities within 1e-12 relative (forward vs recursive association);
  * per-pixel mean XYZ: L2 error < 1e-5 (north_star), weights exact.
C1-C4 compare with the oracle's reference mode (the reference's exhaustive line traversal); C5
with its pruned mode (same closest hit, distance-culled; tests/test_oracle_scene.py checks the two
equal), because the exhaustive walk over a 1M-triangle tree is too slow for a test.
"""
import os

import numpy as np
import pytest

from vanrijn_amd import scenes
from vanrijn_amd.render import Tile, render_samples, render_tile

pytestmark = pytest.mark.gpu

XYZ_L2_TOL = 1e-5          # north_star: per-pixel L2 error < 1e-5 vs reference
INTENSITY_REL_TOL = 1e-12  # forward vs recursive throughput association
SEED = 0x5EED0001
THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


@pytest.fixture(scope="module")
def bunny():
    return scenes.procedural_bunny()


def _decisions_equal(gpu, ref):
    assert np.array_equal(gpu["flags"], ref["flags"])
    assert np.array_equal(gpu["bounces"], ref["bounces"])
    assert np.array_equal(gpu["wavelength"], ref["wavelength"])
    assert np.array_equal(gpu["intensity"] == 0, ref["intensity"] == 0)
    nz = ref["intensity"] != 0
    rel = np.abs(gpu["intensity"][nz] - ref["intensity"][nz]) / np.abs(ref["intensity"][nz])
    assert (rel < INTENSITY_REL_TOL).all(), float(rel.max())


def _check(scene, orc, mode, tile, H, W, spp, band_rows=None):
    """Decisions sample by sample (in row bands, to bound the record memory), then the image."""
    band = band_rows or tile.height()
    hits = 0
    for r0 in range(tile.start_row, tile.end_row, band):
        t = Tile(tile.start_column, tile.end_column, r0, min(tile.end_row, r0 + band))
        ref = orc.render_samples(t, H, W, spp, seed=SEED, mode=mode, nthreads=THREADS)
        gpu = render_samples(scene, t, H, W, spp, seed=SEED)
        _decisions_equal(gpu, ref)
        hits += int((ref["flags"] & 1).sum())
    ref = orc.render_tile(tile, H, W, spp, seed=SEED, mode=mode, nthreads=THREADS)
    gpu = render_tile(scene, tile, H, W, spp, seed=SEED)
    err = np.linalg.norm(gpu.colour_buffer - ref["colour"], axis=2)
    assert err.max() < XYZ_L2_TOL, float(err.max())
    assert np.array_equal(gpu.weight_buffer, ref["weight"])
    assert np.array_equal(gpu.weight_buffer, np.full((tile.height(), tile.width()), float(spp)))
    return hits


def test_c1_bench_scene_full_frame(bunny, oracle):
    s = scenes.bench_scene(bunny)
    hits = _check(s, oracle.OracleScene(s.spec()), oracle.MODE_REFERENCE, Tile(0, 256, 0, 256), 256, 256, 16)
    assert hits > 100_000


def test_c2_main_scene_full_frame(bunny, oracle):
    s = scenes.main_scene(bunny)
    hits = _check(s, oracle.OracleScene(s.spec()), oracle.MODE_REFERENCE, Tile(0, 512, 0, 512), 512, 512, 64,
                  band_rows=64)
    assert hits > 5_000_000


def test_c3_crop_of_1024_frame(bunny, oracle):
    s = scenes.main_scene(bunny)
    hits = _check(s, oracle.OracleScene(s.spec()), oracle.MODE_REFERENCE, Tile(448, 576, 448, 576), 1024, 1024, 32)
    assert hits > 100_000


def test_c4_crop_of_2048_frame(bunny, oracle):
    s = scenes.main_scene(bunny)
    _check(s, oracle.OracleScene(s.spec()), oracle.MODE_REFERENCE, Tile(1000, 1064, 1100, 1164), 2048, 2048, 16)


@pytest.fixture(scope="module")
def c5_pair(oracle):
    s = scenes.synthetic_scene()
    return s, oracle.OracleScene(s.spec())


def test_c5_crop_of_4096_frame(c5_pair, oracle):
    s, orc = c5_pair
    assert s.device_scene(0).info()["triangle_count"] == 1_051_392
    hits = _check(s, orc, oracle.MODE_PRUNED, Tile(1700, 1764, 2200, 2264), 4096, 4096, 4)
    assert hits > 10_000

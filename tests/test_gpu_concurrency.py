"""Concurrent callers on one scene (include/vanrijn_amd.h "Threading"), and per-call errors.

The reference calls partial_render_scene on one shared &Scene from rayon workers
(src/main.rs:197-211).  Here several host threads call through the C ABI at once: each call holds
its own call context (stream, staging buffer, queue counter, error word), so the results must be
exactly the serial results of the same sample indices, and a singular shading basis found by one
call (the reference panics, simple_random_integrator.rs:26-31) must not leak into another.

det == 0 cannot be produced by finite geometry here (every basis is built from normalised, mutually
orthogonal vectors; a degenerate one turns into NaN, which the reference does not treat as
singular either), so the error tests use the library's test-only entry point
vr_debug_set_fault_object: hits on that object take the singular-basis path.
"""
import threading

import numpy as np
import pytest

from vanrijn_amd import _native as N
from vanrijn_amd import records as R
from vanrijn_amd import scenes
from vanrijn_amd.render import (Tile, collect_launch_times, partial_render_scene, render_tile, render_tile_device,
                                stream_check_error)

pytestmark = pytest.mark.gpu

PARTIAL_SEED = 0x5EED0001  # vr_partial_render_scene's stream seed (include/vanrijn_amd.h)


def _run_threads(fn, n):
    out, errs = [None] * n, []

    def work(k):
        try:
            out[k] = fn(k)
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append(e)

    ts = [threading.Thread(target=work, args=(k,)) for k in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    return out


@pytest.fixture(scope="module")
def small_main():
    return scenes.main_scene(scenes.displaced_mesh(16, scenes._BUNNY_BUMPS, 0xB0BB1E, 24, 0.04,
                                                   (1.25, 1.05, 1.15), (-1.7, -0.8, 0.0)))


def test_eight_threads_render_tile_equal_serial(small_main):
    H, W, spp = 48, 64, 2
    t = Tile(0, W, 0, H)
    ds = small_main.device_scene(0)
    par = _run_threads(lambda k: render_tile(ds, t, H, W, spp, seed=11, first_sample=k * spp), 8)
    for k in range(8):
        ser = render_tile(ds, t, H, W, spp, seed=11, first_sample=k * spp)
        for f in ("colour_buffer", "colour_sum_buffer", "colour_bias_buffer", "weight_buffer", "weight_bias_buffer"):
            assert np.array_equal(getattr(par[k], f), getattr(ser, f)), (k, f)


def test_eight_threads_partial_render_scene_union(small_main):
    """32 concurrent 1-spp calls draw pass indices 0..31 from the scene's counter: as a multiset
    the results are the serial renders of sample indices 0..31."""
    H, W = 40, 56
    t = Tile(0, W, 0, H)
    from vanrijn_amd.scene import DeviceScene
    ds = DeviceScene(small_main.spec(), 0)  # a fresh scene: its pass counter starts at 0

    def calls(k):
        return [partial_render_scene(ds, t, H, W) for _ in range(4)]

    got = [b for bs in _run_threads(calls, 8) for b in bs]
    assert all(np.array_equal(b.weight_buffer, np.ones((H, W))) for b in got)
    key = lambda a: a.tobytes()  # noqa: E731
    got_keys = sorted(key(b.colour_sum_buffer) for b in got)
    want_keys = sorted(key(render_tile(ds, t, H, W, 1, seed=PARTIAL_SEED, first_sample=i).colour_sum_buffer)
                       for i in range(32))
    assert got_keys == want_keys


@pytest.fixture(scope="module")
def faulty_scene(small_main, oracle):
    """A second device copy of the scene with the test hook on object 1 (the mesh BVH)."""
    from vanrijn_amd.scene import DeviceScene
    ds = DeviceScene(small_main.spec(), 0)
    ds.set_fault_object(1)
    # rows whose camera rays hit nothing: no shading there, so no fault can occur
    H = W = 64
    ref = oracle.OracleScene(small_main.spec()).render_samples(Tile(0, W, 0, H), H, W, 1, seed=1)
    sky_rows = int(np.argmax((ref["flags"][..., 0] & 1).any(axis=1)))
    assert sky_rows >= 4, sky_rows
    return ds, H, W, sky_rows


def test_singular_basis_is_reported_to_its_own_call(faulty_scene):
    ds, H, W, sky_rows = faulty_scene
    full, sky = Tile(0, W, 0, H), Tile(0, W, 0, sky_rows)

    def call(k):
        try:
            render_tile(ds, full if k % 2 == 0 else sky, H, W, 2, seed=3, first_sample=k)
            return N.VR_OK
        except N.VrError as e:
            return e.code

    codes = _run_threads(call, 8)
    assert codes == [-5, 0] * 4, codes  # VR_ERROR_SINGULAR_BASIS exactly where the mesh is shaded


def test_async_error_sticks_to_its_stream(faulty_scene):
    import torch
    ds, H, W, sky_rows = faulty_scene
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    st1 = torch.zeros(H * W * 8, dtype=torch.float64, device="cuda")
    st2 = torch.zeros(W * sky_rows * 8, dtype=torch.float64, device="cuda")
    # untimed launches return at once; the fault is found later, on the device
    render_tile_device(ds, Tile(0, W, 0, H), H, W, 2, 3, 0, st1.data_ptr(), s1.cuda_stream)
    render_tile_device(ds, Tile(0, W, 0, sky_rows), H, W, 2, 3, 0, st2.data_ptr(), s2.cuda_stream)
    with pytest.raises(N.VrError) as e:
        stream_check_error(ds, s1.cuda_stream)
    assert e.value.code == -5
    stream_check_error(ds, s1.cuda_stream)  # cleared by the check
    stream_check_error(ds, s2.cuda_stream)  # the clean stream never saw it
    # a timed launch reports its own stream's error synchronously
    with pytest.raises(N.VrError):
        render_tile_device(ds, Tile(0, W, 0, H), H, W, 1, 3, 0, st1.data_ptr(), s1.cuda_stream, timed=True)
    torch.cuda.synchronize()


def test_clean_scene_streams_check_ok(small_main):
    import torch
    ds = small_main.device_scene(0)
    s = torch.cuda.Stream()
    st = torch.zeros(32 * 32 * 8, dtype=torch.float64, device="cuda")
    render_tile_device(ds, Tile(0, 32, 0, 32), 32, 32, 2, 3, 0, st.data_ptr(), s.cuda_stream)
    stream_check_error(ds, s.cuda_stream)
    assert float(R.sums(st)[:, 3].sum()) == 2 * 32 * 32


def test_deferred_launch_times(small_main, faulty_scene):
    """VR_LAUNCH_DEFER_TIMES (bench.py's timed frames): the launches queue without a host wait and
    vr_collect_launch_times returns their summed event times once; the records equal timed launches'
    bit for bit; device errors of deferred launches are reported by the collection."""
    import torch
    ds = small_main.device_scene(0)
    s = torch.cuda.Stream()
    t = Tile(0, 64, 0, 64)
    a = torch.zeros(64 * 64 * 8, dtype=torch.float64, device="cuda")
    b = torch.zeros_like(a)
    assert collect_launch_times(ds, s.cuda_stream)["launches"] == 0  # nothing deferred yet
    timed = [render_tile_device(ds, t, 64, 64, 4, 9, 4 * k, a.data_ptr(), s.cuda_stream, accumulate=k > 0,
                                timed=True) for k in range(3)]
    for k in range(3):
        st = render_tile_device(ds, t, 64, 64, 4, 9, 4 * k, b.data_ptr(), s.cuda_stream, accumulate=k > 0,
                                defer_times=True)
        assert st["timed"] == 0 and st["passes"] == 1
    lt = collect_launch_times(ds, s.cuda_stream)
    assert lt["launches"] == 3 and lt["passes"] == 3 and lt["max_passes"] == 1
    assert lt["kernel_ms"] > 0 and lt["reduce_ms"] > 0
    assert all(x["timed"] == 1 and x["kernel_ms"] > 0 for x in timed)
    assert torch.equal(a, b)
    assert collect_launch_times(ds, s.cuda_stream)["launches"] == 0  # collected once
    # a deferred launch's singular basis is reported by the collection, then the stream is clean
    fds, H, W, _ = faulty_scene
    st = torch.zeros(H * W * 8, dtype=torch.float64, device="cuda")
    render_tile_device(fds, Tile(0, W, 0, H), H, W, 1, 3, 0, st.data_ptr(), s.cuda_stream, defer_times=True)
    with pytest.raises(N.VrError) as e:
        collect_launch_times(fds, s.cuda_stream)
    assert e.value.code == -5
    stream_check_error(fds, s.cuda_stream)

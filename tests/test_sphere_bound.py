"""The f32 sphere pre-test's margin (vr_device.h sphere_maybe32_lanes), checked on the CPU.

begin_ray skips the f64 Sphere::intersect (sphere.rs:39-93) when every lane's f32 estimate says
the LINE passes the sphere by more than 1e-4 |oc|^2 + 1e-12 (|o|^2 + |c|^2).  That is only sound if
the reference's f64 discriminant b^2 - 4ac is then negative (the reference returns None).  Here the
f32 arithmetic is emulated exactly (numpy float32 operations round each operation to nearest, like
the kernel built with -ffp-contract=off) and the f64 discriminant follows sphere.rs's operation
order, on rays built to graze the sphere (relative offsets 1e-9 .. 1e-1, both sides, origins near
and far).  Every "missed" verdict must have a negative discriminant.
"""
import numpy as np

F32 = np.float32


def missed32(o, d, c, r):
    ox, oy, oz = (F32(o[:, k] - c[:, k]) for k in range(3))
    dx, dy, dz = (d[:, k].astype(F32) for k in range(3))
    t = ox * dx + oy * dy + oz * dz
    oc2 = ox * ox + oy * oy + oz * oz
    rf = r.astype(F32)
    o32 = o.astype(F32)
    c32 = c.astype(F32)
    po = o32[:, 0] * o32[:, 0] + o32[:, 1] * o32[:, 1] + o32[:, 2] * o32[:, 2]
    pc = c32[:, 0] * c32[:, 0] + c32[:, 1] * c32[:, 1] + c32[:, 2] * c32[:, 2]
    return (oc2 - t * t) - rf * rf > F32(1e-4) * oc2 + F32(1e-12) * (po + pc)


def discriminant(o, d, c, r):
    """sphere.rs:43-59: a, b, c from component products, folded from 0.0; b^2 - 4ac."""
    a = ((0.0 + d[:, 0] * d[:, 0]) + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
    bv = 2.0 * (o * d - c * d)
    b = ((0.0 + bv[:, 0]) + bv[:, 1]) + bv[:, 2]
    cv = (o * o + c * c) - 2.0 * (c * o)
    cc = ((0.0 + cv[:, 0]) + cv[:, 1]) + cv[:, 2]
    cc = cc - r * r
    return b * b - 4.0 * a * cc


def _grazing(rng, n, scale, far):
    c = rng.uniform(-scale, scale, (n, 3))
    r = rng.uniform(0.05, 3.0, n)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    p = rng.normal(size=(n, 3))
    p -= (p * d).sum(1, keepdims=True) * d
    p /= np.linalg.norm(p, axis=1, keepdims=True)
    rel = 10.0 ** rng.uniform(-9, -1, n) * rng.choice([-1.0, 1.0], n)
    s = rng.uniform(-far, far, n)
    o = c + p * (r * (1.0 + rel))[:, None] + d * s[:, None]
    return o, d, c, r


def test_missed_implies_negative_discriminant():
    rng = np.random.default_rng(0x5EED)
    total_skips = 0
    for scale, far in ((10.0, 20.0), (10.0, 1e3), (1e3, 50.0), (1.0, 5.0)):
        o, d, c, r = _grazing(rng, 200_000, scale, far)
        m = missed32(o, d, c, r)
        delta = discriminant(o, d, c, r)
        assert (delta[m] < 0.0).all(), np.flatnonzero(m & ~(delta < 0.0))[:5]
        total_skips += int(m.sum())
    assert total_skips > 30_000  # the margin still lets clear misses (rel >~ 1e-4) be skipped


def test_clear_misses_and_hits():
    rng = np.random.default_rng(7)
    o, d, c, r = _grazing(rng, 10_000, 10.0, 20.0)
    # lines at 1.5 r: skipped; lines through the centre: never skipped
    d2 = d.copy()
    p = rng.normal(size=d.shape)
    p -= (p * d2).sum(1, keepdims=True) * d2
    p /= np.linalg.norm(p, axis=1, keepdims=True)
    far_o = c + p * (1.5 * r)[:, None] + d2 * rng.uniform(-5, 5, (len(r), 1))
    assert missed32(far_o, d2, c, r).all()
    centre_o = c + d2 * rng.uniform(-5, 5, (len(r), 1))
    assert not missed32(centre_o, d2, c, r).any()

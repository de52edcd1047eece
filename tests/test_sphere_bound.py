"""The f32 sphere pre-test's margin (vr_device.h sphere_missed32), checked on the CPU.

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


def skip32(o, d, c, r, best):
    """vr_device.h sphere_skip32: line miss, sphere behind the origin, or near root beyond best."""
    ox, oy, oz = (F32(o[:, k] - c[:, k]) for k in range(3))
    dx, dy, dz = (d[:, k].astype(F32) for k in range(3))
    t = ox * dx + oy * dy + oz * dz
    rf = r.astype(F32)
    o32 = o.astype(F32)
    c32 = c.astype(F32)
    m = (F32(1e-4) * (np.abs(ox) + np.abs(oy) + np.abs(oz)) +
         F32(1e-6) * (np.abs(o32[:, 0]) + np.abs(o32[:, 1]) + np.abs(o32[:, 2]) +
                      np.abs(c32[:, 0]) + np.abs(c32[:, 1]) + np.abs(c32[:, 2]) + rf))
    b32 = best.astype(F32)
    with np.errstate(invalid="ignore", over="ignore"):
        behind = t - rf > m
        beyond = (-t - rf) - m > b32 + F32(1e-6) * np.abs(b32) + F32(1e-30)
    return missed32(o, d, c, r) | behind | beyond


def sphere_distance(o, d, c, r):
    """sphere.rs:39-93 in its operation order: the distance, or NaN for None."""
    a = ((0.0 + d[:, 0] * d[:, 0]) + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
    bv = 2.0 * (o * d - c * d)
    b = ((0.0 + bv[:, 0]) + bv[:, 1]) + bv[:, 2]
    cv = (o * o + c * c) - 2.0 * (c * o)
    cc = ((0.0 + cv[:, 0]) + cv[:, 1]) + cv[:, 2]
    cc = cc - r * r
    ds = b * b - 4.0 * a * cc
    with np.errstate(invalid="ignore"):
        delta = np.sqrt(ds)
    inv = 1.0 / (2.0 * a)
    t1 = (-b - delta) * inv
    t2 = (-b + delta) * inv
    dist = np.where((t1 < 0.0) | ((t2 >= 0.0) & (t1 >= t2)), t2, t1)
    return np.where((ds < 0.0) | ~(dist > 0.0), np.nan, dist)


def test_skip_implies_no_closer_hit():
    """A skipped sphere returns None or a distance that does not beat `best` (dd < best fails)."""
    rng = np.random.default_rng(0xB0B)
    skips = {"behind": 0, "beyond": 0}
    for scale, far in ((10.0, 20.0), (10.0, 1e3), (1e3, 50.0), (1.0, 5.0)):
        o, d, c, r = _grazing(rng, 200_000, scale, far)
        dist = sphere_distance(o, d, c, r)
        # best distances straddling the sphere's near root: 1e-9 .. 1e-1 relative, both sides
        near = np.where(np.isnan(dist), np.abs(rng.normal(size=len(r))) * far, dist)
        rel = 10.0 ** rng.uniform(-9, -1, len(r)) * rng.choice([-1.0, 1.0], len(r))
        best = np.maximum(near * (1.0 + rel), 0.0)
        best[rng.random(len(r)) < 0.1] = np.inf
        s = skip32(o, d, c, r, best)
        bad = s & ~np.isnan(dist) & (dist < best)
        assert not bad.any(), np.flatnonzero(bad)[:5]
        skips["behind"] += int((s & ~missed32(o, d, c, r) & np.isnan(dist)).sum())
        skips["beyond"] += int((s & ~np.isnan(dist)).sum())
    assert skips["behind"] > 10_000 and skips["beyond"] > 2_000, skips


def test_skip_behind_and_beyond_cases():
    rng = np.random.default_rng(11)
    n = 10_000
    c = rng.uniform(-10, 10, (n, 3))
    r = rng.uniform(0.1, 2.0, n)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    inf = np.full(n, np.inf)
    # origin 3 r in front of the centre along d: the sphere is behind, skipped
    o = c + d * (3.0 * r)[:, None]
    assert skip32(o, d, c, r, inf).all()
    # origin 3 r before the centre, looking at it: a hit at 2 r, never skipped unless best < 2 r
    o = c - d * (3.0 * r)[:, None]
    assert not skip32(o, d, c, r, inf).any()
    assert not skip32(o, d, c, r, 2.0 * r * (1 + 1e-3)).any()
    assert skip32(o, d, c, r, 1.9 * r).all()
    # origin inside the sphere: never behind
    o = c + d * (0.5 * r)[:, None]
    assert not skip32(o, d, c, r, inf).any()

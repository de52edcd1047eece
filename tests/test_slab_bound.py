"""The f32 box pre-test's error bound (vr_device.h slab32 / prepare32), checked on the CPU.

The kernel decides most box tests in f32: slab values t = fma(b32, i32, -(o32 * i32)) on the
outward-rounded box, error margin E = ek + 3e-7 (|lo| + |hi|), ek = 6e-7 (max(extent, |o|) + 1)
max|i32| (since round 4 the kernel uses the per-ray constant E = 3.001 ek, which bounds that margin
for every box within the scene extent: checked case by case here); it answers "hit" only if
hi - lo > 2E, "miss" only if lo - hi > 2E, and otherwise re-runs
the reference's f64 division test (raycasting/axis_aligned_bounding_box.rs:9-27).  Here the f32
arithmetic is emulated exactly (numpy float32 operations are IEEE round-to-nearest; the fma is
formed in float64 from exact float32 products and rounded once) on rays and boxes built to sit on
or near a tie, and every f32 verdict must equal the f64 division verdict.  The kernel's reciprocals
are the hardware's v_rcp_f32 (within 1 ulp of 1/d, not correctly rounded): the test also takes,
per axis at random, either f32 neighbour of the exact reciprocal.
"""
import numpy as np

F32 = np.float32


def f64_slab(b, o, d):
    lo, hi = -np.inf, np.inf
    with np.errstate(divide="ignore", invalid="ignore"):
        for a in range(3):
            x = (b[2 * a] - o[a]) / d[a]
            y = (b[2 * a + 1] - o[a]) / d[a]
            mn, mx = (y, x) if x > y else (x, y)
            lo = np.fmax(lo, mn)
            hi = np.fmin(hi, mx)
    return not (lo > hi)


def outward(b):
    out = np.empty(6, dtype=F32)
    for k in range(6):
        f = F32(b[k])
        if k % 2 == 0 and float(f) > b[k]:
            f = np.nextafter(f, F32(-np.inf))
        if k % 2 == 1 and float(f) < b[k]:
            f = np.nextafter(f, F32(np.inf))
        out[k] = f
    return out


def fma32(a, b, c):
    return F32(np.float64(a) * np.float64(b) + np.float64(c))  # exact product, one rounding of the sum
                                                               # in f64, then to f32 (double rounding
                                                               # is below the bound's slack)


def recip32(d32, rng=None):
    """1 / d32 correctly rounded, or (rng given) either f32 neighbour of the exact value: what a
    1-ulp reciprocal may return"""
    with np.errstate(divide="ignore", over="ignore", invalid="ignore"):
        rn = (F32(1.0) / d32).astype(F32)
        if rng is None:
            return rn
        out = rn.copy()
        for a in range(3):
            exact = 1.0 / np.float64(d32[a]) if d32[a] != 0 else np.inf
            if not np.isfinite(exact) or not np.isfinite(rn[a]):
                continue
            down = rn[a] if float(rn[a]) <= exact else np.nextafter(rn[a], F32(-np.inf))
            up = rn[a] if float(rn[a]) >= exact else np.nextafter(rn[a], F32(np.inf))
            out[a] = down if rng.random() < 0.5 else up
        return out


def f32_slab(b32, o, d, extent, rcp_rng=None, const_margin=False):
    o32 = o.astype(F32)
    i32 = recip32(d.astype(F32), rcp_rng)
    with np.errstate(divide="ignore", over="ignore", invalid="ignore"):
        n32 = -(o32 * i32)
    big = max(extent, float(np.abs(o).max())) + 1.0
    ek = 6e-7 * big * float(np.abs(i32).max())
    ek = F32(ek) if ek < 1e30 else F32(np.inf)
    t = [fma32(b32[k], i32[k // 2], n32[k // 2]) for k in range(6)]
    lo = max(min(t[0], t[1]), min(t[2], t[3]), min(t[4], t[5]))
    hi = min(max(t[0], t[1]), max(t[2], t[3]), max(t[4], t[5]))
    e = F32(ek + F32(3e-7) * (abs(lo) + abs(hi)))
    if const_margin:
        # the kernel's form since round 4: E = 3.001 ek per ray (vr_device.h Ray32), which bounds the
        # per-box margin above for every box of the scene; one difference, two compares
        e2 = 2.0 * (3.001 * (6e-7 * big * float(np.abs(i32).max())))
        # round_away_f32: (float)t times 1 + 2^-22, rounded (at least t)
        E2 = F32(F32(e2) * F32(1.0 + 2.0 ** -22)) if e2 < 1e30 else F32(np.inf)
        assert float(E2) >= e2
        assert float(E2) >= 2.0 * float(e), (float(E2), float(e))
        dd = F32(lo - hi)
        if dd < -E2:
            return 1
        if dd > E2:
            return 0
        return 2
    if F32(hi - lo) > F32(2.0) * e:
        return 1
    if F32(lo - hi) > F32(2.0) * e:
        return 0
    return 2


import pytest  # noqa: E402


@pytest.mark.parametrize("const_margin", [False, True])
@pytest.mark.parametrize("rcp", ["rn", "1ulp"])
def test_f32_pretest_never_contradicts_the_exact_test(rcp, const_margin):
    rng = np.random.default_rng(5)
    rcp_rng = np.random.default_rng(11) if rcp == "1ulp" else None
    extent = 8.0
    decided = undecided = 0
    for _ in range(20000):
        o = rng.uniform(-extent, extent, 3)
        d = rng.normal(size=3)
        if rng.random() < 0.2:  # near-axis directions: large 1/d
            d[rng.integers(3)] *= 10.0 ** -rng.integers(2, 7)
        d /= np.linalg.norm(d)
        # a box with one face through a point on the line (a near tie), or a random box
        t = rng.uniform(-5, 5)
        p = o + t * d
        lo = np.minimum(p - rng.exponential(0.5, 3), p + rng.normal(0, 1e-6, 3))
        hi = np.maximum(p + rng.exponential(0.5, 3), lo)
        k = rng.integers(3)
        if rng.random() < 0.5:  # put the line exactly on / just off a face
            lo[k] = p[k] + rng.choice([0.0, 1e-12, -1e-12, 1e-7, -1e-7])
            hi[k] = max(hi[k], lo[k])
        b = np.array([lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]])
        b = np.clip(b, -extent, extent)
        b[1::2] = np.maximum(b[1::2], b[0::2])
        r = f32_slab(outward(b), o, d, extent, rcp_rng, const_margin)
        exact = f64_slab(b, o, d)
        if r == 2:
            undecided += 1
        else:
            decided += 1
            assert bool(r) == exact, (b, o, d)
    assert decided > 0.8 * (decided + undecided)  # the pre-test decides most cases

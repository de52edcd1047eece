"""normalize_n1 (vr_device.h): the reciprocal norm of a near-unit vector from the bits of x = a.a.

normalize (vec3.rs:103-110) multiplies by 1 / sqrt(a.a).  For x within 4096 spacings of 1.0 the
kernel takes 1 / sqrt(x) from integer arithmetic on x's bits instead of the f64 sqrt and division
sequences (DESIGN.md "Near-unit normalisation").  Here every x the kernel's range admits (and 16x
more on either side, the margin of the second-order argument) is checked against the correctly
rounded 1.0 / sqrt(x) of IEEE f64 (numpy), bit for bit.
"""
import numpy as np

ONE = np.int64(0x3FF0000000000000)


def inv_norm_near1(b):
    """The kernel's formula: b = bits(x) - bits(1.0) -> bits of 1 / sqrt(x)."""
    b = np.asarray(b, dtype=np.int64)
    j = np.where(b >= 0, b >> 1, (1 - b) >> 1)
    r = np.where(b >= 0, ONE - 2 * j, ONE + ((j + 1) >> 1))
    return r.view(np.float64)


def test_every_admitted_square_norm_bitwise():
    b = np.arange(-65536, 65537, dtype=np.int64)
    x = (ONE + b).view(np.float64)
    want = 1.0 / np.sqrt(x)
    got = inv_norm_near1(b)
    assert np.array_equal(got.view(np.int64), want.view(np.int64)), b[got != want][:8]


def test_normalised_vectors_land_in_the_range():
    """Unit vectors rebuilt from unit vectors: their a.a (folded from -0.0 like vec3.rs:76-82)
    lies within a few spacings of 1, far inside the kernel's +-4096."""
    rng = np.random.default_rng(5)
    v = rng.normal(size=(200_000, 3))
    inv = 1.0 / np.sqrt(((-0.0 + v[:, 0] * v[:, 0]) + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2])
    u = v * inv[:, None]
    x = ((-0.0 + u[:, 0] * u[:, 0]) + u[:, 1] * u[:, 1]) + u[:, 2] * u[:, 2]
    b = x.view(np.int64) - ONE
    assert np.abs(b).max() <= 16
    # and the fast path's normalisation equals normalize's
    got = u * inv_norm_near1(b)[:, None]
    want = u * (1.0 / np.sqrt(x))[:, None]
    assert np.array_equal(got, want)


def test_sphere_a_of_normalised_directions_lands_in_the_range():
    """a = ((0 + dx dx) + dy dy) + dz dz (sphere.rs:43-47, fold from 0.0) of the kernel's ray
    directions (normalize / normalize_n1 of arbitrary vectors) lies within a few spacings of 1."""
    rng = np.random.default_rng(9)
    v = rng.normal(size=(200_000, 3)) * rng.uniform(1e-3, 1e3, size=(200_000, 1))
    inv = 1.0 / np.sqrt(((-0.0 + v[:, 0] * v[:, 0]) + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2])
    d = v * inv[:, None]
    a = ((0.0 + d[:, 0] * d[:, 0]) + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
    assert np.abs(a.view(np.int64) - ONE).max() <= 16

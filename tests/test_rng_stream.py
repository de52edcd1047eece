"""The counter-based random stream "vr-hash32 v2" (DESIGN.md section 3), on the CPU.

The reference draws from rand 0.7's ThreadRng, which cannot be seeded; the oracle and
the kernels share this stream instead, and the parity tests compare them on it.  Here:
  * the oracle's stream (oracle/vr_oracle.c orc_stream_base / orc_stream_draw) equals an independent
    pure-Python restatement of the spec, on fixed and random (seed, pixel, sample, draw) -- the same
    spec the kernel implements (vr_device.h Rng), which the GPU parity tests then pin bit for bit;
  * statistical sanity of what the path consumes: the 53-bit Standard values are uniform (chi-square
    over 1024 bins), consecutive draws of a sample -- the camera's (x, y) jitter, the Lambertian
    rejection pairs -- are uniform as pairs (chi-square over a 32 x 32 grid) and uncorrelated, the
    draw's high and low words are uncorrelated, neighbouring pixels' and samples' streams are
    uncorrelated, and the Lambertian rejection loop accepts a pair with probability pi / 4.
  * parity of the u64 -> f64 maps with rand 0.7 is not pinned here (test_oracle_kats.py restates them).
"""
import numpy as np

M64 = (1 << 64) - 1
M32 = (1 << 32) - 1
SALT = 0x76616E52696A6E31


def mix64(z):
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def hash32(x):
    x &= M32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & M32
    return x ^ (x >> 16)


def stream_base(seed, pixel, sample):
    return mix64(mix64(seed ^ SALT) ^ (((pixel << 32) + sample) & M64))


def stream_draw(base, k):
    x = ((base & M32) + (k + 1) * 0x9E3779B9) & M32
    v = x ^ (base >> 32)
    return (hash32(v) << 32) | hash32(v + 0x6A09E667)


def test_oracle_stream_matches_the_spec(oracle):
    L = oracle.lib()
    assert L.orc_hash32(0) == 0 and L.orc_hash32(1) == hash32(1)
    rng = np.random.default_rng(3)
    cases = [(0x5EED0001, 0, 0), (0x5EED0001, 1023 * 1024 + 511, 255), (7, 10, 3), ((1 << 64) - 1, (1 << 32) - 1, 5)]
    cases += [(int(rng.integers(0, 1 << 62)), int(rng.integers(0, 1 << 24)), int(rng.integers(0, 4096)))
              for _ in range(50)]
    for seed, pixel, sample in cases:
        b = stream_base(seed, pixel, sample)
        assert L.orc_stream_base(seed, pixel, sample) == b
        for k in (0, 1, 2, 7, 1000, 123456):
            assert L.orc_stream_draw(b, k) == stream_draw(b, k), (seed, pixel, sample, k)
    for x in rng.integers(0, 1 << 32, 200):
        assert L.orc_hash32(int(x)) == hash32(int(x))


def _draws(L, n_samples, n_draws, seed=0x5EED0001):
    """[sample][draw] 64-bit draws of consecutive pixels' sample 0..: n_samples streams."""
    out = np.empty((n_samples, n_draws), dtype=np.uint64)
    for i in range(n_samples):
        b = L.orc_stream_base(seed, i // 4, i % 4)
        for k in range(n_draws):
            out[i, k] = L.orc_stream_draw(b, k)
    return out


def _chi2_ok(counts):
    """chi-square of uniform counts within 5 standard deviations of its mean (df = bins - 1)."""
    counts = np.asarray(counts, dtype=np.float64).ravel()
    e = counts.sum() / counts.size
    chi2 = ((counts - e) ** 2 / e).sum()
    df = counts.size - 1
    return abs(chi2 - df) < 5 * np.sqrt(2 * df), chi2


def test_stream_statistics(oracle):
    L = oracle.lib()
    d = _draws(L, 4096, 24)
    u = (d >> np.uint64(11)).astype(np.float64) * 2.0 ** -53  # rand 0.7 Standard
    ok, chi2 = _chi2_ok(np.histogram(u, bins=1024, range=(0, 1))[0])
    assert ok, chi2
    # consecutive draws of a sample as pairs (camera jitter x, y; Lambertian rejection pairs)
    a, b = u[:, 0::2].ravel(), u[:, 1::2].ravel()
    ok, chi2 = _chi2_ok(np.histogram2d(a, b, bins=32, range=[[0, 1], [0, 1]])[0])
    assert ok, chi2
    lim = 5.0 / np.sqrt(a.size)
    assert abs(np.corrcoef(a, b)[0, 1]) < lim
    # high and low words of one draw
    hi = (d >> np.uint64(32)).astype(np.float64).ravel()
    lo = (d & np.uint64(0xFFFFFFFF)).astype(np.float64).ravel()
    assert abs(np.corrcoef(hi, lo)[0, 1]) < 5.0 / np.sqrt(hi.size)
    # neighbouring streams: pixel p and p + 1 (same sample), sample s and s + 1 (same pixel), draw by draw
    pix = u.reshape(1024, 4, 24)
    for x, y in ((pix[:-1, 0], pix[1:, 0]), (pix[:, 0], pix[:, 1])):
        assert abs(np.corrcoef(x.ravel(), y.ravel())[0, 1]) < 5.0 / np.sqrt(x.size)
    # every bit of the 64 is fair
    bits = np.array([((d >> np.uint64(i)) & np.uint64(1)).mean() for i in range(64)])
    assert (np.abs(bits - 0.5) < 5 * 0.5 / np.sqrt(d.size)).all(), bits


def test_lambertian_rejection_acceptance(oracle):
    """lambertian_material.rs:36-49: pairs (2 Open01 - 1)^2 summed <= 1 with probability pi / 4."""
    L = oracle.lib()
    d = _draws(L, 2048, 32)
    o = np.array([[L.orc_u64_to_open01(int(v)) for v in row] for row in d])
    x, y = 2.0 * o[:, 0::2] - 1.0, 2.0 * o[:, 1::2] - 1.0
    acc = (x * x + y * y <= 1.0).mean()
    n = x.size
    assert abs(acc - np.pi / 4) < 5 * np.sqrt(np.pi / 4 * (1 - np.pi / 4) / n), acc

// vr_device.h -- device-side building blocks of the gfx950 path tracer (included by vr_render.hip).
//
// f64 vector math, the counter-based random stream, spectra and CIE matching, the reference's
// exact line-slab test, ray-triangle / sphere / plane tests, closest-hit traversal and hit
// shading data.  Every expression follows the operation order of the reference's Rust source
// (file:line cited per function) and is compiled with -ffp-contract=off, so decisions are
// bit-identical to the oracle.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vanrijn_amd.h"
#include "rgb_spectrum_tables.h"
#include "vr_layout.h"

namespace vr {
namespace dev {

// ----------------------------------------------------------------------------------------------
// f64 vector helpers in the reference's operation order (src/math/vec3.rs)
// ----------------------------------------------------------------------------------------------
struct V3 {
    double x, y, z;
};
__device__ __forceinline__ V3 mk(double x, double y, double z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 scl(V3 a, double s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 neg(V3 a) { return mk(-a.x, -a.y, -a.z); }
// vec3.rs:76-82 -- `Sum for f64` folds from -0.0
__device__ __forceinline__ double dot(V3 a, V3 b) {
    double s = -0.0;
    s = s + a.x * b.x;
    s = s + a.y * b.y;
    s = s + a.z * b.z;
    return s;
}
__device__ __forceinline__ V3 cross(V3 a, V3 b) {  // vec3.rs:84-89
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ V3 normalize(V3 a) {  // vec3.rs:103-110 (multiply by 1/norm)
    double inv = 1.0 / sqrt(dot(a, a));
    return mk(a.x * inv, a.y * inv, a.z * inv);
}
// normalize for vectors whose squared norm x lies within 4096 spacings of 1.0 (unit vectors
// rebuilt from unit vectors: a second normalisation, orthonormal-basis transforms, the tangent of
// two orthogonal unit vectors), with the same bits as normalize.  With u = 2^-52:
//   x = 1 + k u (k >= 0):      sqrt(x) = 1 + k u/2 - k^2 u^2/8 ...  rounds to s = 1 + floor(k/2) u,
//                              and 1/s = 1 - j u + j^2 u^2 ...       rounds to 1 - 2j (u/2);
//   x = 1 - k u/2 (k > 0):     sqrt(x) = 1 - k u/4 - k^2 u^2/32 ... rounds to s = 1 - ceil(k/2) u/2,
//                              and 1/s = 1 + j u/2 + j^2 u^2/4 ...   rounds to 1 + ceil(j/2) u
// (the second-order terms are nonzero and far below half a spacing for |k| <= 2^16, so they only
// break the ties the first-order values sit on).  On the bits: b = bits(x) - bits(1.0) is k above
// 1 and -k below.  Every such x is checked against the correctly rounded 1 / sqrt(x) in
// tests/test_normalize_near1.py; other lanes take normalize's sqrt and division.
// every active lane's b (bits of a.a minus bits of 1.0) within +-4096: one unsigned 64-bit compare
// into a lane mask (llvm.amdgcn.icmp; a ballot of the two signed tests is lowered to two compares,
// a v_cndmask and a v_cmp)
__device__ __forceinline__ bool near1_all(int64_t b) {
    return __builtin_amdgcn_uicmpl((uint64_t)(b + 4096), 8192ull, 34 /* ugt */) == 0;
}
__device__ __forceinline__ V3 normalize_n1(V3 a) {
    const double x = dot(a, a);
    const int64_t one = 0x3FF0000000000000ll;
    const int64_t b = __double_as_longlong(x) - one;
    double inv;
    // wave-uniform: the whole wave takes the bit formula or the sqrt and division (a divergent
    // branch would be if-converted into both)
    if (near1_all(b)) {
        const int64_t j = b >= 0 ? (b >> 1) : ((1 - b) >> 1);  // s = 1 + j u  or  1 - j u/2
        inv = __longlong_as_double(b >= 0 ? one - 2 * j : one + ((j + 1) >> 1));
    } else {
        inv = 1.0 / sqrt(x);
    }
    return mk(a.x * inv, a.y * inv, a.z * inv);
}
__device__ __forceinline__ bool sgn(double x) { return __double_as_longlong(x) < 0; }
__device__ __forceinline__ double sel(V3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }
__device__ __forceinline__ V3 ldv(const double* p) { return mk(p[0], p[1], p[2]); }

// ----------------------------------------------------------------------------------------------
// Random stream "vr-hash32 v2" + rand 0.7 maps (same definition as oracle/vr_oracle.c; DESIGN.md
// section 3).  Per (pixel, sample) one 64-bit base, mix64(key ^ (pixel << 32 | sample)), then draw k
// hashes a 32-bit Weyl counter (base's low word + k * 0x9E3779B9) xored with base's high word twice
// with Wellons' lowbias32 -- 12 VALU (4 of them v_mul_lo_u32) per 64-bit draw, against 17 (a 64-bit
// xorshift-multiply finaliser: 3 v_lshrrev_b64, 2 v_mad_u64_u32, 4 v_mul_lo_u32) for splitmix64's
// finaliser per draw and two per base in round 4's "vr-splitmix v1" (draw mixing measured at 7.6 %
// of the C3 launch's VALU instructions, profiles/r05/rng).
// ----------------------------------------------------------------------------------------------
constexpr uint64_t kSeedSalt = 0x76616E52696A6E31ull;
constexpr uint32_t kWeyl32 = 0x9E3779B9u;
constexpr uint32_t kLoOffset = 0x6A09E667u;
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint32_t hash32(uint32_t x) {  // lowbias32
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}
struct Rng {
    uint32_t x, y;  // the draw counter (base's low word + k * kWeyl32 after k draws) and base's high word
    __device__ __forceinline__ void reset(uint64_t base) {
        x = (uint32_t)base;
        y = (uint32_t)(base >> 32);
    }
    __device__ __forceinline__ uint64_t next() {
        x += kWeyl32;
        const uint32_t v = x ^ y;
        return ((uint64_t)hash32(v) << 32) | hash32(v + kLoOffset);
    }
    // rand 0.7 Standard f64 (camera.rs:49, photon.rs:21)
    __device__ __forceinline__ double standard() { return (double)(next() >> 11) * 0x1.0p-53; }
    // rand 0.7 Open01 f64 (lambertian_material.rs:39-48)
    __device__ __forceinline__ double open01() {
        return __longlong_as_double((long long)((next() >> 12) | 0x3FF0000000000000ull)) - (1.0 - 0x1.0p-53);
    }
    // rand 0.7 Standard bool, `(next_u32() as i32) < 0` (smooth_transparent_dialectric.rs:103):
    // the u32 is the draw's high half, so the bool is the draw's top bit
    __device__ __forceinline__ bool boolean() { return (int32_t)(uint32_t)(next() >> 32) < 0; }
};
// the stream base from seed_key = mix64(seed ^ kSeedSalt) (a per-launch constant, RenderArgs::seed_key)
__device__ __forceinline__ uint64_t stream_base_keyed(uint64_t seed_key, uint64_t pixel, uint64_t sample) {
    return mix64(seed_key ^ ((pixel << 32) + sample));
}

// ----------------------------------------------------------------------------------------------
// Spectra (src/colour/spectrum.rs) and CIE matching (colour_xyz.rs:86-103)
// ----------------------------------------------------------------------------------------------
__constant__ double c_rgbspec[7][32] = VR_RGBSPEC_BASIS_INIT;

// Spectrum::intensity_at_wavelength (spectrum.rs:64-79); sample(j) supplies samples[j]
template <class F>
__device__ __forceinline__ double spectrum_at(double shortest, double longest, int n, double wl, F sample) {
    if (wl < shortest || wl > longest) return 0.0;
    double range = longest - shortest;
    int i = (int)((double)(n - 1) * ((wl - shortest) / range));  // `as usize` (wl >= shortest here)
    double before = (double)i / (double)(n - 1) * range + shortest;
    if (i == n - 1) return sample(i);
    double after = (double)(i + 1) / (double)(n - 1) * range + shortest;
    double delta = after - before;
    double ratio = (wl - before) / delta;
    return sample(i) * (1.0 - ratio) + sample(i + 1) * ratio;
}

__device__ __forceinline__ double material_colour(const Material* m, double wl) {
    return spectrum_at(m->shortest, m->longest, m->n, wl, [&](int j) { return m->samples[j]; });
}

// The same lookup for values that are only intensities (a BSDF's colour, the sky, light
// spectra): the segment index from one multiplication (at a knot either neighbour gives the same
// value to rounding) and the knots from the host's table (the reference's values bit for bit);
// one division (the ratio) instead of four.  Within 1e-15 relative of spectrum_at; never used
// where the value steers a ray (the dielectric's eta keeps material_colour).
template <class F>
__device__ __forceinline__ double spectrum_fast(const Material* m, double wl, F sample) {
    if (wl < m->shortest || wl > m->longest) return 0.0;
    const int n = m->n;
    int i = (int)((wl - m->shortest) * m->inv_step);
    i = i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
    if (i == n - 1) return sample(i);
    const double before = m->knots[i], after = m->knots[i + 1];
    const double ratio = (wl - before) / (after - before);
    return sample(i) * (1.0 - ratio) + sample(i + 1) * ratio;
}
__device__ __forceinline__ double material_intensity(const Material* m, double wl) {
    return spectrum_fast(m, wl, [&](int j) { return m->samples[j]; });
}

// ----------------------------------------------------------------------------------------------
// Phong and dielectric materials (materials/phong_material.rs, smooth_transparent_dialectric.rs)
// ----------------------------------------------------------------------------------------------
constexpr double kPi = 3.14159265358979323846;  // std::f64::consts::PI

// Material::sample's default, CosineWeightedHemisphere::value (cosine_weighted_hemisphere.rs:20-
// 29) over UnitDisc (unit_disc.rs:28-40, Shirley's concentric map) over UniformSquare
// (uniform_square.rs:21-26: corner + (Open01, Open01) * size, x drawn first)
__device__ __forceinline__ V3 cosine_weighted_hemisphere(Rng& rng) {
    const double ux = rng.open01();
    const double uy = rng.open01();
    const double ox = -1.0 + ux * 2.0, oy = -1.0 + uy * 2.0;
    double px = ox, py = oy;
    if (!(ox == 0.0 && oy == 0.0)) {
        double radius, angle;
        if (fabs(ox) > fabs(oy)) {
            radius = ox;
            angle = ((kPi / 4.0) * oy) / ox;
        } else {
            radius = oy;
            angle = kPi / 2.0 - ((kPi / 4.0) * ox) / oy;
        }
        px = cos(angle) * radius;
        py = sin(angle) * radius;
    }
    const double z = sqrt(fmax(0.0, 1.0 - px * px - py * py));
    return mk(px, py, z);
}
__device__ __forceinline__ double cosine_weighted_pdf(V3 v) { return sqrt(v.x * v.x + v.y * v.y) / kPi; }

// fresnel (smooth_transparent_dialectric.rs:15-62)
struct Fresnel {
    V3 rdir, tdir;
    double R, T;
};
__device__ __forceinline__ Fresnel fresnel(V3 w_i, double eta1, double eta2) {
    Fresnel f;
    const V3 normal = w_i.z > 0.0 ? mk(0.0, 0.0, 1.0) : mk(-0.0, -0.0, -1.0);  // -Vec3::unit_z()
    f.rdir = mk(-w_i.x, -w_i.y, w_i.z);
    const double r = eta1 / eta2;
    const double c1 = dot(normal, w_i);
    const double c2sq = 1.0 - r * r * (1.0 - c1 * c1);
    if (c2sq >= 0.0) {
        const double c2 = sqrt(c2sq);
        const double rpar = (eta1 * c2 - eta2 * c1) / (eta1 * c2 + eta2 * c1);
        const double rper = (eta1 * c1 - eta2 * c2) / (eta1 * c1 + eta2 * c2);
        f.R = 0.5 * (rpar * rpar + rper * rper);
        const double k = r * c1 - c2;
        f.tdir = normalize(add(mk(-r * w_i.x, -r * w_i.y, -r * w_i.z), mk(k * normal.x, k * normal.y, k * normal.z)));
        f.T = 1.0 - f.R;
    } else {
        f.R = 1.0;
        f.T = 0.0;
        f.tdir = mk(0.0, 0.0, 0.0);
    }
    if (w_i.z < 0.0) {
        f.rdir.z *= -1.0;
        f.tdir.z *= -1.0;
    }
    return f;
}
// eta pair by side (smooth_transparent_dialectric.rs:81-86,94-99)
__device__ __forceinline__ Fresnel dielectric_fresnel(const Material* m, V3 w_i, double wl) {
    const double eta = material_colour(m, wl);
    return w_i.z >= 0.0 ? fresnel(w_i, 1.0, eta) : fresnel(w_i, eta, 1.0);
}
// the bsdf's strength for an outgoing direction (smooth_transparent_dialectric.rs:88-95)
__device__ __forceinline__ double dielectric_strength(const Fresnel& f, V3 w_o) {
    const V3 dr = sub(w_o, f.rdir);
    if (dot(dr, dr) < 0.0000000001) return f.R;
    const V3 dt = sub(w_o, f.tdir);
    if (dot(dt, dt) < 0.0000000001) return f.T;
    return 0.0;
}

// test_lighting_environment (simple_random_integrator.rs:57-65): reflection_from_linear_rgb of
// (w.y, w.y, 1) (spectrum.rs:81-165), evaluated only at the two samples the lookup needs.
__device__ double sky_intensity(double wy, double wl, const Material* knots) {
    const double r = wy, g = wy, b = 1.0;
    double c0, c1, c2;
    int kx, ky;
    if (r <= g && r <= b) {
        if (g <= b) { c0 = r; c1 = g - r; c2 = b - g; kx = VR_RGBSPEC_CYAN; ky = VR_RGBSPEC_BLUE; }
        else { c0 = r; c1 = b - r; c2 = g - b; kx = VR_RGBSPEC_CYAN; ky = VR_RGBSPEC_GREEN; }
    } else if (g <= r && g < b) {
        if (r <= b) { c0 = g; c1 = r - g; c2 = b - r; kx = VR_RGBSPEC_MAGENTA; ky = VR_RGBSPEC_BLUE; }
        else { c0 = g; c1 = b - g; c2 = r - b; kx = VR_RGBSPEC_MAGENTA; ky = VR_RGBSPEC_RED; }
    } else {
        if (r <= g) { c0 = b; c1 = r - b; c2 = g - r; kx = VR_RGBSPEC_YELLOW; ky = VR_RGBSPEC_GREEN; }
        else { c0 = b; c1 = g - b; c2 = r - g; kx = VR_RGBSPEC_YELLOW; ky = VR_RGBSPEC_RED; }
    }
    return spectrum_fast(knots, wl, [&](int j) {
        return c0 * c_rgbspec[VR_RGBSPEC_WHITE][j] + c1 * c_rgbspec[kx][j] + c2 * c_rgbspec[ky][j];
    });
}

__device__ __forceinline__ double gaussian(double wl, double alpha, double mu, double s1, double s2) {
    double s = wl < mu ? s1 : s2;
    double denominator = 2.0 * (s * s);
    double t = wl - mu;
    return alpha * exp(-(t * t) / denominator);
}
// The ordered reduce's form: exp(-(t^2) * k) with k = 1 / (2 s^2) a compile-time constant per lobe
// side instead of a division per lobe, and the table-driven exp (vr_exp_table.h, within 2 ulp of
// exp): the colour is an output value only, within 1e-14 relative of xyz_for_wavelength.
// `tab` holds VR_EXP_TABLE_INIT (the reduce keeps it in LDS)
__device__ __forceinline__ double gaussian_kt(double wl, double alpha, double mu, double k1, double k2,
                                              const double* tab) {
    const double k = wl < mu ? k1 : k2;
    const double t = wl - mu;
    return alpha * vr_exp_tab(-(t * t) * k, tab);
}
#define VR_GT(alpha, mu, s1, s2) \
    gaussian_kt(wl, alpha, mu, 1.0 / (2.0 * ((s1) * (s1))), 1.0 / (2.0 * ((s2) * (s2))), tab)
__device__ __forceinline__ V3 xyz_for_wavelength_tab(double wl, const double* tab) {
    return mk(VR_GT(1.056, 599.8, 37.9, 31.0) + VR_GT(0.362, 442.0, 16.0, 26.7) + VR_GT(-0.065, 501.1, 20.4, 26.2),
              VR_GT(0.821, 568.8, 46.9, 40.5) + VR_GT(0.286, 530.9, 16.3, 31.1),
              VR_GT(1.217, 437.0, 11.8, 36.0) + VR_GT(0.681, 459.0, 26.0, 13.8));
}
#undef VR_GT
__device__ __forceinline__ V3 xyz_for_wavelength(double wl) {
    return mk(gaussian(wl, 1.056, 599.8, 37.9, 31.0) + gaussian(wl, 0.362, 442.0, 16.0, 26.7) +
                  gaussian(wl, -0.065, 501.1, 20.4, 26.2),
              gaussian(wl, 0.821, 568.8, 46.9, 40.5) + gaussian(wl, 0.286, 530.9, 16.3, 31.1),
              gaussian(wl, 1.217, 437.0, 11.8, 36.0) + gaussian(wl, 0.681, 459.0, 26.0, 13.8));
}

// ----------------------------------------------------------------------------------------------
// Rays and primitives
// ----------------------------------------------------------------------------------------------
struct Ray {
    V3 o, d;
};
// Per-ray constants hoisted out of every box / triangle test (bit-identical to recomputing them)
struct RayPre {
    V3 o, d;
    double sx, sy, pdz;
    int flags;  // bits 0-1: axis rotation r (permutation [r, r+1, r+2] mod 3); bit 2: exact_only
                // (some |d_i| tiny or zero: every slab takes the division path); bit 3: behind_ok
                // (|shear-axis component| >= 0.01: boxes behind the origin may be culled)
    __device__ __forceinline__ int k0() const { return flags & 3; }
    __device__ __forceinline__ int k1() const { int k = (flags & 3) + 1; return k == 3 ? 0 : k; }
    __device__ __forceinline__ int k2() const { int k = (flags & 3) + 2; return k >= 3 ? k - 3 : k; }
    __device__ __forceinline__ bool exact_only() const { return (flags & 4) != 0; }
    __device__ __forceinline__ bool behind_ok() const { return (flags & 8) != 0; }
};

__device__ __forceinline__ RayPre prepare(const Ray& r) {
    RayPre p;
    p.o = r.o;
    p.d = r.d;
    // indices_with_index_of_largest_element_last (triangle.rs:108-122): signed comparisons;
    // the three outcomes [0,1,2], [1,2,0], [2,0,1] are the rotations r = 0, 1, 2
    int rot;
    if (r.d.x > r.d.y) rot = (r.d.z > r.d.x) ? 0 : 1;
    else rot = (r.d.z > r.d.y) ? 0 : 2;
    const int k0 = rot, k1 = rot == 2 ? 0 : rot + 1, k2 = rot == 0 ? 2 : rot - 1;
    double pdx = sel(r.d, k0), pdy = sel(r.d, k1), pdz = sel(r.d, k2);
    p.sx = -pdx / pdz;  // calculate_shear_to_z_axis (triangle.rs:129-131)
    p.sy = -pdy / pdz;
    p.pdz = pdz;
    const double tiny = 1e-150;
    const bool exact_only = !(fabs(r.d.x) > tiny && fabs(r.d.y) > tiny && fabs(r.d.z) > tiny);
    p.flags = rot | (exact_only ? 4 : 0) | (fabs(pdz) >= 0.01 ? 8 : 0);
    return p;
}

// raycasting/axis_aligned_bounding_box.rs:9-27 (+ util/interval.rs): the LINE slab test with
// NaN-ignoring max/min, in the reference's division form (the exact decision).  Only called
// where the f32 test cannot decide (slab32 == 2) and on the test-only / shadow-ray paths.
// tlo / thi: the line interval, for distance culling.
__device__ __forceinline__ bool slab(const double* b, const RayPre& p, double& tlo, double& thi) {
    double elo = -INFINITY, ehi = INFINITY;
    {
        double a = (b[0] - p.o.x) / p.d.x, c = (b[1] - p.o.x) / p.d.x;
        double mn = a > c ? c : a, mx = a > c ? a : c;
        elo = fmax(elo, mn); ehi = fmin(ehi, mx);
    }
    {
        double a = (b[2] - p.o.y) / p.d.y, c = (b[3] - p.o.y) / p.d.y;
        double mn = a > c ? c : a, mx = a > c ? a : c;
        elo = fmax(elo, mn); ehi = fmin(ehi, mx);
    }
    {
        double a = (b[4] - p.o.z) / p.d.z, c = (b[5] - p.o.z) / p.d.z;
        double mn = a > c ? c : a, mx = a > c ? a : c;
        elo = fmax(elo, mn); ehi = fmin(ehi, mx);
    }
    tlo = elo;
    thi = ehi;
    return !(elo > ehi);
}

// f32 pre-decision of the line slab test on an outward-rounded f32 box.  Returns 1 (the exact
// f64 test passes), 0 (it fails) or 2 (too close to call: run the exact test).  tlo/thi are
// conservative: the exact interval lies within [tlo, thi] when 1 is returned.
// Error bound (DESIGN.md "Traversal"): with |bound|, |origin| <= X (scene extent or |o|), each f32
// slab value differs from the exact (bound - o)/d by at most ~3e-7 X |1/d_i| + 1.2e-7 |t|
// (outward box rounding, f32 origin, subtraction, reciprocal and product roundings); E doubles it.
struct Ray32 {
    float ox, oy, oz, ix, iy, iz;
    float nx, ny, nz;  // -(o * inv) per axis (f32): slab values are fma(bound, inv, n)
    float e2;  // 2 E, E = 3.001 ek >= every box's ek + 3e-7 (|lo| + |hi|) (+inf: every test falls back to f64)
};
// The margin as one per-ray constant (round 4).  The bound per box was E_box = ek + 3e-7 (|lo| + |hi|)
// with ek = 6e-7 X m (X = max(extent, |o|) + 1, m = max_i |1/d_i|).  Every slab value is
// fma(b, i, -(o i)) with |b| <= extent (the scene's coordinates bound every box, rounded outward by
// at most 2^-23 relative) and |o| <= X - 1, so |t| <= 2 X m (1 + 2^-22); lo and hi are slab values,
// hence 3e-7 (|lo| + |hi|) <= 1.2e-6 X m (1 + 2^-22) = 2 ek (1 + 2^-22), and E_box (its f32 evaluation
// included) < 3.001 ek = E.  A decision taken with E is taken with E_box too, so it inherits that
// bound's soundness (tests/test_slab_bound.py checks both); it saves the per-box margin arithmetic
// (|lo| + |hi|, the fma, lo - e, hi + e, 2e) in the node step, and the cull thresholds carry E.
// an f32 at least as far from 0 as t (a normal or infinite t): (float)t is within 2^-24 relative of t,
// and one product by 1 + 2^-22 (rounded) moves it beyond -- one multiply instead of a compare and
// nextafterf.  Used for the cull thresholds (t >= margin > 0 away from +0, or t <= -behind_margin)
// and the margin itself, where a wider value is only more conservative.
__device__ __forceinline__ float round_away_f32(double t) { return (float)t * (1.0f + 0x1p-22f); }
__device__ __forceinline__ Ray32 prepare32(const RayPre& p, double extent) {
    Ray32 r;
    r.ox = (float)p.o.x; r.oy = (float)p.o.y; r.oz = (float)p.o.z;
    // hardware f32 reciprocals of the f32 direction (v_rcp_f32: within 1 ulp, 1.2e-7 relative, of
    // 1/d -- the bound's reciprocal term; tests/test_slab_bound.py takes either f32 neighbour of the
    // exact value).  |d| = 1, so some |1/d_i| >= 1 and no reciprocal is denormal; a denormal or
    // zero d_i gives an infinite or huge reciprocal, ek = +inf, and every test takes the f64 path
    r.ix = __builtin_amdgcn_rcpf((float)p.d.x);
    r.iy = __builtin_amdgcn_rcpf((float)p.d.y);
    r.iz = __builtin_amdgcn_rcpf((float)p.d.z);
    r.nx = -(r.ox * r.ix); r.ny = -(r.oy * r.iy); r.nz = -(r.oz * r.iz);
    // origins on the infinite plane can lie outside the scene extent: bound with |o| too
    const double big = fmax(extent, fmax(fmax(fabs(p.o.x), fabs(p.o.y)), fabs(p.o.z))) + 1.0;
    const double m = fmax(fmax(fabsf(r.ix), fabsf(r.iy)), fabsf(r.iz));
    const double ek = 6e-7 * big * m;
    r.e2 = (p.exact_only() || !(ek < 1e30)) ? INFINITY : round_away_f32(2.0 * (3.001 * ek));
    return r;
}
// E (half of e2; exact), for the cull thresholds
__device__ __forceinline__ double margin_of(const Ray32& r) { return 0.5 * (double)r.e2; }
// Each slab value is one fused multiply-add per bound, two bounds per packed (v_pk_fma_f32)
// instruction: t = RN(b32 * i32 - RN(o32 * i32)).  Its error against the exact (b - o) / d is at
// most 1.8e-7 |t| + 2.4e-7 X |1/d| (reciprocal of the f32 direction 1.2e-7, fma 6e-8;
// outward-rounded bound 2^-23 |b|, f32 origin and the product o * i 2^-24 each), which
// E_box = ek + 3e-7 (|lo| + |hi|) covers (ek = 6e-7 X max |1/d|); the per-ray E >= E_box (above).
// lo / hi are returned as computed: the exact interval lies within [lo - E, hi + E], and the cull
// thresholds the callers compare them with are widened by E (cull_far + E rounded up, cull_behind -
// E rounded down), so `lo > cull_far'` implies lo - E > cull_far.
typedef float vr_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int slab32(const float* b, const Ray32& r, float& lo, float& hi) {
    const vr_f2 bx = {b[0], b[1]}, by = {b[2], b[3]}, bz = {b[4], b[5]};
    const vr_f2 tx = __builtin_elementwise_fma(bx, (vr_f2){r.ix, r.ix}, (vr_f2){r.nx, r.nx});
    const vr_f2 ty = __builtin_elementwise_fma(by, (vr_f2){r.iy, r.iy}, (vr_f2){r.ny, r.ny});
    const vr_f2 tz = __builtin_elementwise_fma(bz, (vr_f2){r.iz, r.iz}, (vr_f2){r.nz, r.nz});
    lo = fmaxf(fmaxf(fminf(tx.x, tx.y), fminf(ty.x, ty.y)), fminf(tz.x, tz.y));
    hi = fminf(fminf(fmaxf(tx.x, tx.y), fmaxf(ty.x, ty.y)), fmaxf(tz.x, tz.y));
    // lo - hi is exactly -(hi - lo) (round to nearest): both tests on one difference; NaN: 2
    const float d = lo - hi;
    if (d < -r.e2) return 1;
    if (d > r.e2) return 0;
    return 2;
}
// slab32 as two flags (the node step's form, no integer result to re-test): `maybe` = the exact
// test may pass (slab32 != 0; also for a NaN difference), `sure` = it certainly passes (slab32 == 1)
__device__ __forceinline__ void slab32_flags(const float* b, const Ray32& r, float& lo, float& hi, bool& maybe,
                                             bool& sure) {
    const vr_f2 bx = {b[0], b[1]}, by = {b[2], b[3]}, bz = {b[4], b[5]};
    const vr_f2 tx = __builtin_elementwise_fma(bx, (vr_f2){r.ix, r.ix}, (vr_f2){r.nx, r.nx});
    const vr_f2 ty = __builtin_elementwise_fma(by, (vr_f2){r.iy, r.iy}, (vr_f2){r.ny, r.ny});
    const vr_f2 tz = __builtin_elementwise_fma(bz, (vr_f2){r.iz, r.iz}, (vr_f2){r.nz, r.nz});
    lo = fmaxf(fmaxf(fminf(tx.x, tx.y), fminf(ty.x, ty.y)), fminf(tz.x, tz.y));
    hi = fminf(fminf(fmaxf(tx.x, tx.y), fmaxf(ty.x, ty.y)), fmaxf(tz.x, tz.y));
    const float d = lo - hi;
    sure = d < -r.e2;
    maybe = !(d > r.e2);
}

// A triangle record in one batch of five dwordx4 loads.  Left to itself the scheduler issued the
// last vertex's z only after the first four loads had returned (two memory round trips per
// triangle test); the empty asm needs all five values at once, so all five are in flight together.
__device__ __forceinline__ TriVerts load_tri(const TriVerts* p) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const u4* q = reinterpret_cast<const u4*>(p);
    u4 w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4];
    asm volatile("" : "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3), "+v"(w4));
    const u4 w[5] = {w0, w1, w2, w3, w4};
    TriVerts t;
    __builtin_memcpy(&t, w, sizeof t);
    return t;
}

// Triangle::intersect decision part (triangle.rs:35-66): returns distance, or -1 on a miss
// (a valid hit's distance is a norm, >= 0).  Vertices are translated by -origin (v + (-o) ==
// v - o bitwise), permuted so the ray's largest signed component is last, sheared (z unscaled).
__device__ __forceinline__ double triangle_distance(const TriVerts& t, const RayPre& p, double bary[3]) {
    const int k0 = p.k0(), k1 = p.k1(), k2 = p.k2();
    double tx[3], ty[3], az[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        // translated in the scene's axes, then permuted: sel(v + (-o), k) is sel(v, k) + (-sel(o, k))
        // bit for bit, and the origin needs no selects of its own (12 v_cndmask per test)
        const V3 a = mk(t.v[3 * i] + (-p.o.x), t.v[3 * i + 1] + (-p.o.y), t.v[3 * i + 2] + (-p.o.z));
        const double ax = sel(a, k0), ay = sel(a, k1);
        az[i] = sel(a, k2);
        tx[i] = ax + p.sx * az[i];
        ty[i] = ay + p.sy * az[i];
    }
    // signed_edge_functions (triangle.rs:141-158): e0 = E(v1, v2), e1 = E(v2, v0), e2 = E(v0, v1)
    const double e0 = tx[1] * ty[2] - tx[2] * ty[1];
    const double e1 = tx[2] * ty[0] - tx[0] * ty[2];
    const double e2 = tx[0] * ty[1] - tx[1] * ty[0];
    const bool s0 = sgn(e0), s1 = sgn(e1), s2 = sgn(e2);
    if (!((!s0 && !s1 && !s2) || (s0 && s1 && s2))) return -1.0;
    const double ea0 = fabs(e0), ea1 = fabs(e1), ea2 = fabs(e2);
    double s = 0.0;  // fold(0.0) (triangle.rs:160-162)
    s = s + ea0;
    s = s + ea1;
    s = s + ea2;
    const double inv = 1.0 / s;
    const double b0 = ea0 * inv, b1 = ea1 * inv, b2 = ea2 * inv;
    double tz = 0.0;  // explicit fold(0.0) (triangle.rs:57-61)
    tz = tz + az[0] * b0;
    tz = tz + az[1] * b1;
    tz = tz + az[2] * b2;
    if (sgn(tz) != sgn(p.pdz)) return -1.0;
    // fold(Vec3::zeros()) (triangle.rs:66-71) without its first `0 +`: 0 + x differs from x only when
    // x is -0 (+0), so the sums below differ from the reference's at most in the sign of a zero,
    // which o - loc and the squares of the norm erase (o - (+-0) == o for o != 0; (+-0)^2 == +0):
    // the distance's bits are the reference's (the hit location itself is recomputed for shading)
    V3 loc = scl(mk(t.v[0], t.v[1], t.v[2]), b0);
    loc = add(loc, scl(mk(t.v[3], t.v[4], t.v[5]), b1));
    loc = add(loc, scl(mk(t.v[6], t.v[7], t.v[8]), b2));
    const V3 dv = sub(p.o, loc);
    bary[0] = b0;
    bary[1] = b1;
    bary[2] = b2;
    return sqrt(dot(dv, dv));
}

// sphere.rs:43-47's a = sum of d * d (fold from 0.0) -- the same for every sphere a ray meets
__device__ __forceinline__ double sphere_a(V3 d) {
    double a = 0.0;
    a = a + d.x * d.x;
    a = a + d.y * d.y;
    a = a + d.z * d.z;
    return a;
}
// Sphere::intersect (sphere.rs:39-93), decision part: distance or -1; `a` = sphere_a(p.d) and
// `one_over_2_a` = 1 / (2a) of the ray, hoisted out of the loop over spheres (the same bits)
__device__ __forceinline__ double sphere_distance(const Prim& s, const RayPre& p, double a, double one_over_2_a) {
    V3 o = p.o, d = p.d, c = ldv(s.vec);
    V3 bv = scl(sub(mk(o.x * d.x, o.y * d.y, o.z * d.z), mk(c.x * d.x, c.y * d.y, c.z * d.z)), 2.0);
    double b = 0.0;
    b = b + bv.x;
    b = b + bv.y;
    b = b + bv.z;
    V3 cv = sub(add(mk(o.x * o.x, o.y * o.y, o.z * o.z), ldv(s.pre)),  // s.pre: c * c per component
                scl(mk(c.x * o.x, c.y * o.y, c.z * o.z), 2.0));
    double cc = 0.0;
    cc = cc + cv.x;
    cc = cc + cv.y;
    cc = cc + cv.z;
    cc = cc - s.scalar2;  // radius * radius
    double delta_squared = b * b - 4.0 * a * cc;
    if (delta_squared < 0.0) return -1.0;
    double delta = sqrt(delta_squared);
    double t1 = (-b - delta) * one_over_2_a;
    double t2 = (-b + delta) * one_over_2_a;
    double distance = (t1 < 0.0 || (t2 >= 0.0 && t1 >= t2)) ? t2 : t1;
    if (distance <= 0.0) return -1.0;
    return distance;
}

// Conservative f32 pre-test for Sphere::intersect: the sphere is ruled out ("missed") only if the
// LINE passes it so far outside that the reference's f64 discriminant b^2 - 4ac is certainly
// negative (the call returns None).  In exact arithmetic delta = 4|d|^2 (r^2 - dist^2), dist^2 = |oc|^2 - (oc.d)^2 / |d|^2;
// the f64 evaluation errs by O(1e-16 (|o|^2 + |c|^2 + |oc|^2)) and this f32 estimate of
// dist^2 - r^2 by < 2e-6 |oc|^2 (|d| = 1 +- 1e-16; conversions, products and sums each 6e-8
// relative), so the margin 1e-4 |oc|^2 + 1e-12 (|o|^2 + |c|^2) covers both.  NaN: not missed.
// the lanes (of the active ones) for which the pre-test cannot rule the sphere out, as one v_cmp:
// !(lhs > rhs) is "unordered or less-equal"
__device__ __forceinline__ uint64_t sphere_maybe32_lanes(const Prim& s, const RayPre& p) {
    const float ox = (float)(p.o.x - s.vec[0]), oy = (float)(p.o.y - s.vec[1]), oz = (float)(p.o.z - s.vec[2]);
    const float dx = (float)p.d.x, dy = (float)p.d.y, dz = (float)p.d.z;
    const float t = ox * dx + oy * dy + oz * dz;
    const float oc2 = ox * ox + oy * oy + oz * oz;
    const float r = (float)s.scalar;
    const float po = (float)p.o.x * (float)p.o.x + (float)p.o.y * (float)p.o.y + (float)p.o.z * (float)p.o.z;
    const float pc = (float)s.vec[0] * (float)s.vec[0] + (float)s.vec[1] * (float)s.vec[1] +
                     (float)s.vec[2] * (float)s.vec[2];
    return __builtin_amdgcn_fcmpf((oc2 - t * t) - r * r, 1e-4f * oc2 + 1e-12f * (po + pc), 13 /* ule */);
}

// Plane::intersect (plane.rs:49-75): t or -1 (t == 0 is a hit).  NaN t (ray inside the plane)
// is reported as a hit with NaN distance, as in the reference; it never wins a comparison here.
__device__ __forceinline__ bool plane_distance(const Prim& pl, const RayPre& p, double& t) {
    V3 n = ldv(pl.vec);
    double dn = dot(p.d, n);
    const V3 q = ldv(pl.pre);  // normal * distance
    double num = dot(sub(q, p.o), n);
    if (dn == 0.0) {
        if (num != 0.0) return false;
    }
    t = num / dn;
    return !(t < 0.0);
}

struct HitInfo {
    V3 loc, normal, tangent, cotangent, retro;
    int material;
};


// triangle_distance's barycentrics only (the winning triangle's shading, whose hit is known):
// the same operations up to b0..b2, without tz, the location and the distance's sqrt
__device__ __forceinline__ void triangle_bary(const TriVerts& t, const RayPre& p, double bary[3]) {
    const int k0 = p.k0(), k1 = p.k1(), k2 = p.k2();
    double tx[3], ty[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {  // translated, then permuted (as triangle_distance)
        const V3 a = mk(t.v[3 * i] + (-p.o.x), t.v[3 * i + 1] + (-p.o.y), t.v[3 * i + 2] + (-p.o.z));
        const double ax = sel(a, k0), ay = sel(a, k1);
        const double az = sel(a, k2);
        tx[i] = ax + p.sx * az;
        ty[i] = ay + p.sy * az;
    }
    const double ea0 = fabs(tx[1] * ty[2] - tx[2] * ty[1]);
    const double ea1 = fabs(tx[2] * ty[0] - tx[0] * ty[2]);
    const double ea2 = fabs(tx[0] * ty[1] - tx[1] * ty[0]);
    double s = 0.0;
    s = s + ea0;
    s = s + ea1;
    s = s + ea2;
    const double inv = 1.0 / s;
    bary[0] = ea0 * inv;
    bary[1] = ea1 * inv;
    bary[2] = ea2 * inv;
}

// full Triangle::intersect for the winning triangle (shading data: triangle.rs:66-96).  `dist` (the
// hit's distance, sqrt((o - loc).(o - loc)) over the same loc bits) is not needed: the retro direction
// is normalised like the reference (dividing by `dist` instead gives the same bits but measured no
// faster, round 2's VR_RETRO_DIST)
__device__ void triangle_info(const TriVerts& t, const TriNormals& nn, const RayPre& p, double dist, HitInfo& h) {
    double b[3];
    triangle_bary(t, p, b);
    V3 v0 = mk(t.v[0], t.v[1], t.v[2]), v1 = mk(t.v[3], t.v[4], t.v[5]), v2 = mk(t.v[6], t.v[7], t.v[8]);
    V3 loc = mk(0.0, 0.0, 0.0);
    loc = add(loc, scl(v0, b[0]));
    loc = add(loc, scl(v1, b[1]));
    loc = add(loc, scl(v2, b[2]));
    V3 ns = mk(0.0, 0.0, 0.0);
    ns = add(ns, scl(mk(nn.n[0], nn.n[1], nn.n[2]), b[0]));
    ns = add(ns, scl(mk(nn.n[3], nn.n[4], nn.n[5]), b[1]));
    ns = add(ns, scl(mk(nn.n[6], nn.n[7], nn.n[8]), b[2]));
    V3 n = normalize(ns);
    V3 cot = normalize(cross(sub(v0, v1), n));
    h.loc = loc;
    h.normal = n;
    h.cotangent = cot;
    h.tangent = normalize_n1(cross(cot, n));  // cot, n: orthogonal unit vectors
    h.retro = normalize(sub(p.o, loc));
}

__device__ void prim_info(const Prim& pr, const RayPre& p, double dist, HitInfo& h) {
    h.material = pr.material;
    if (pr.kind == 0) {  // plane.rs:66-74
        h.loc = add(p.o, scl(p.d, dist));
        h.normal = ldv(pr.vec);
        h.tangent = ldv(pr.tan);
        h.cotangent = ldv(pr.cot);
        h.retro = neg(p.d);
    } else {  // sphere.rs:71-90
        V3 loc = add(p.o, scl(p.d, dist));
        V3 n = normalize_n1(sub(loc, ldv(pr.vec)));  // |loc - c| = r: near 1 for unit spheres
        V3 tan = normalize(cross(n, mk(0.0, 0.0, 1.0)));
        h.loc = loc;
        h.normal = n;
        h.tangent = tan;
        h.cotangent = cross(n, tan);
        h.retro = neg(p.d);
    }
}

// ----------------------------------------------------------------------------------------------
// Closest hit (sampler.rs:9-20 over vec_aggregate.rs:11-45 and bounding_volume_hierarchy.rs:77-120)
// ----------------------------------------------------------------------------------------------
enum HitKind : int { kNone = 0, kPrim = 1, kTri = 2 };
struct Best {
    double d;
    int kind;
    int index;   // prim index, or global leaf-ordered triangle index
    int object;  // scene object index (ties between objects: the earlier object wins, min_by)
    uint32_t rank;  // a triangle's reference rank (TriVerts::rank; ties within a BVH: the higher wins)
    double bary[3];
};

struct Counts {
    uint32_t box_tests, node_visits, tri_tests, rays, shaded;
    uint32_t trav_slots, outer_slots;  // wave-level loop iterations x 64 (counted by one lane)
    uint32_t exact_boxes;              // f32 box tests too close to call (f64 fallback)
};
__device__ __forceinline__ bool first_active_lane() {
    return __lane_id() == (unsigned)__builtin_ctzll(__ballot(1));
}

template <int STACK, bool COUNT>
__device__ __forceinline__ void traverse_bvh(const DeviceScene& S, const Bvh& bvh, const RayPre& p, Best& best,
                                             int* st_node, float* st_t, int tid, Counts& cnt) {
    if (bvh.root == INT32_MIN) return;  // empty mesh: the reference's empty leaf never hits
    const double margin = S.margin;
    const double behind = S.behind_margin;
    auto cull = [&](double tlo, double thi) {
        double bound = best.kind ? best.d : INFINITY;
        if (tlo > bound + margin * (1.0 + fabs(bound))) return true;
        if (p.behind_ok() && thi < -behind) return true;
        return false;
    };
    // triangle candidate: distance ties go to the later leaf within this BVH (closest_intersection
    // keeps `b` unless a.distance < b.distance, bounding_volume_hierarchy.rs:85) and to the
    // earlier object across objects.
    auto test_tri = [&](int tri) {  // global leaf-ordered triangle index
        if (COUNT) cnt.tri_tests++;
        double b[3];
        double d = triangle_distance(S.tris[tri], p, b);
        if (d < 0.0) return;
        // closest_intersection / min_by (the render kernel's takes_hit): branch-free on the kept rank
        const uint32_t rk = (uint32_t)S.tris[tri].rank;
        const bool closer = !best.kind | (d < best.d);
        const bool tie = (d == best.d) & ((best.object == bvh.object) ? (rk > best.rank) : (bvh.object < best.object));
        if (closer | tie) {
            best.d = d;
            best.kind = kTri;
            best.index = tri;
            best.rank = rk;
            best.object = bvh.object;
            best.bary[0] = b[0];
            best.bary[1] = b[1];
            best.bary[2] = b[2];
        }
    };
    double tlo, thi;
    if (COUNT) cnt.box_tests++;
    if (!slab(bvh.root_box, p, tlo, thi) || cull(tlo, thi)) return;
    if (bvh.root < 0) {
        test_tri(~bvh.root);
        return;
    }
    int node = bvh.root;
    int sp = 0;
    while (true) {
        const Node& nd = S.nodes[node];
        if (COUNT) {
            cnt.node_visits++;
            cnt.box_tests += 2;
            if (first_active_lane()) cnt.trav_slots += 64;
        }
        double lo0, hi0, lo1, hi1;
        const int c0 = nd.child[0], c1 = nd.child[1];
        bool h0 = slab(nd.box[0], p, lo0, hi0) && !cull(lo0, hi0);
        bool h1 = slab(nd.box[1], p, lo1, hi1) && !cull(lo1, hi1);
        if (h0 && c0 < 0) { test_tri(~c0); h0 = false; }
        if (h1 && c1 < 0) { test_tri(~c1); h1 = false; }
        if (h0 && h1) {
            int near = c0, far = c1;
            double far_t = lo1;
            if (lo1 < lo0) { near = c1; far = c0; far_t = lo0; }
            st_node[sp * 256 + tid] = far;
            st_t[sp * 256 + tid] = __double2float_rd(far_t);
            ++sp;
            node = near;
            continue;
        }
        if (h0) { node = c0; continue; }
        if (h1) { node = c1; continue; }
        // pop, skipping entries the (possibly improved) best has since culled
        bool found = false;
        while (sp > 0) {
            --sp;
            double t = (double)st_t[sp * 256 + tid];
            double bound = best.kind ? best.d : INFINITY;
            if (t > bound + margin * (1.0 + fabs(bound))) continue;
            node = st_node[sp * 256 + tid];
            found = true;
            break;
        }
        if (!found) break;
    }
}

template <int STACK, bool COUNT>
__device__ __forceinline__ Best closest_hit(const DeviceScene& S, const RayPre& p, int* st_node, float* st_t, int tid,
                                            Counts& cnt) {
    Best best;
    best.kind = kNone;
    best.d = 0.0;
    best.index = -1;
    best.rank = 0;
    best.object = 0x7fffffff;
    if (COUNT) cnt.rays++;
    // primitive lists, in object then position order: a later equal distance never wins (min_by)
    for (int i = 0; i < S.prim_count; ++i) {
        const Prim& pr = S.prims[i];
        double d;
        bool ok;
        if (pr.kind == 0) ok = plane_distance(pr, p, d);
        else {
            const double a = sphere_a(p.d);
            d = sphere_distance(pr, p, a, 1.0 / (2.0 * a));
            ok = d >= 0.0;
        }
        if (!ok) continue;
        bool take = !best.kind || d < best.d;  // NaN never replaces, never gets replaced
        if (take) {
            best.d = d;
            best.kind = kPrim;
            best.index = i;
            best.object = pr.object;
        }
    }
    for (int b = 0; b < S.bvh_count; ++b) traverse_bvh<STACK, COUNT>(S, S.bvhs[b], p, best, st_node, st_t, tid, cnt);
    return best;
}

// Sampler::sample(shadow ray).is_some() (whitted_integrator.rs:37-38): any object hit.  A
// triangle counts when the exact line test passes on its own box (its leaf) and its test hits --
// ancestors then pass too (superset boxes), so any tree may be walked; no distance ordering is
// needed.  Uses the caller's LDS stack column (`st[depth * 256 + tid]`).
template <int STACK>
__device__ bool any_hit(const DeviceScene& S, const RayPre& p, uint32_t* st, int tid) {
    for (int i = 0; i < S.prim_count; ++i) {
        const Prim& pr = S.prims[i];
        double d;
        if (pr.kind == 0) {
            if (plane_distance(pr, p, d)) return true;
        } else if (sphere_distance(pr, p, sphere_a(p.d), 1.0 / (2.0 * sphere_a(p.d))) >= 0.0) {
            return true;
        }
    }
    for (int b = 0; b < S.bvh_count; ++b) {
        const Bvh& bvh = S.bvhs[b];
        if (bvh.root == INT32_MIN) continue;
        double lo, hi, bary[3];
        if (!slab(bvh.root_box, p, lo, hi)) continue;
        if (bvh.root < 0) {
            if (triangle_distance(S.tris[~bvh.root], p, bary) >= 0.0) return true;
            continue;
        }
        int sp = 0, node = bvh.root;
        while (true) {
            const Node& nd = S.nodes[node];
            int next = -1;
            for (int c = 0; c < 2; ++c) {
                if (!slab(nd.box[c], p, lo, hi)) continue;
                const int ch = nd.child[c];
                if (ch < 0) {
                    if (triangle_distance(S.tris[~ch], p, bary) >= 0.0) return true;
                } else if (next < 0) {
                    next = ch;
                } else {
                    st[sp * 256 + tid] = (uint32_t)ch;
                    ++sp;
                }
            }
            if (next >= 0) {
                node = next;
            } else if (sp > 0) {
                --sp;
                node = (int)st[sp * 256 + tid];
            } else {
                break;
            }
        }
    }
    return false;
}

// Material::bsdf as an affine map of the incoming intensity: out = a * I + b, for the
// WhittedIntegrator's calls (bsdf(w_o, w_i, photon)); lambertian_material.rs:27-34,
// reflective_material.rs:15-40, phong_material.rs:17-36, smooth_transparent_dialectric.rs:79-95
__device__ __forceinline__ void bsdf_affine(const Material* m, V3 w_o, V3 w_i, double wl, double& a, double& b) {
    b = 0.0;
    if (m->kind == 1) {
        if (w_i.z <= 0.0 || w_o.z <= 0.0) {
            a = 0.0;
            return;
        }
        const V3 refl = mk(-w_o.x, -w_o.y, w_o.z);
        double c = dot(w_i, refl);
        c = c < 0.0 ? 0.0 : (c > 1.0 ? 1.0 : c);
        const double theta = acos(fabs(c));
        const double sigma = 0.05, two = 2.0;
        const double f = m->reflection * exp(-(pow(theta, two)) / (two * sigma * sigma));
        a = (material_intensity(m, wl) * m->diffuse) * (1.0 - f);
        b = f;
    } else if (m->kind == 2) {
        if (w_i.z < 0.0 || w_o.z < 0.0) {
            a = 0.0;
            return;
        }
        const V3 refl = mk(-w_i.x, -w_i.y, w_i.z);
        a = material_intensity(m, wl) * m->diffuse;
        b = pow(fabs(dot(w_o, refl)), m->smoothness) * (m->reflection / dot(w_i, mk(0.0, 0.0, 1.0)));
    } else if (m->kind == 3) {
        a = dielectric_strength(dielectric_fresnel(m, w_i, wl), w_o);
    } else {
        a = material_intensity(m, wl) * m->diffuse;
    }
}

__device__ __forceinline__ void hit_info(const DeviceScene& S, const Best& best, const RayPre& p, HitInfo& h) {
    if (best.kind == kPrim) {
        prim_info(S.prims[best.index], p, best.d, h);
    } else {
        triangle_info(S.tris[best.index], S.normals[best.index], p, best.d, h);
        // material of the owning mesh
        int m = 0;
        for (int b = 0; b < S.bvh_count; ++b)
            if (best.object == S.bvhs[b].object) m = S.bvhs[b].material;
        h.material = m;
    }
}

}  // namespace dev
}  // namespace vr

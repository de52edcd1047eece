/*
 * vr_oracle.c -- CPU restatement of vanrijn's per-pixel hot path.  TEST INFRASTRUCTURE ONLY
 * (checker for the MI355X path; see vr_oracle.h for who may load it and what is pinned).
 *
 * Every function cites the reference file:line it restates.  Operation order follows the Rust
 * text exactly (no FMA: built with -ffp-contract=off), because one flipped hit/miss decision
 * moves a pixel by O(1)/spp.
 *
 * "reference" mode is the reference's algorithm: recursive BVH descent into BOTH children of
 * every node whose box the infinite line crosses (bounding_volume_hierarchy.rs:94-120) and the
 * recursive SimpleRandomIntegrator (simple_random_integrator.rs:12-55).  "pruned" mode keeps the
 * same closest-hit semantics but culls subtrees by distance with a conservative margin; it is
 * checked against reference mode in tests/test_oracle_scene.py and exists only to make large
 * CPU comparisons affordable.
 */
#include "vr_oracle.h"
#include "rgb_spectrum_tables.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ======================================================================================== */
/* Random stream "vr-hash32 v2" (replaces rand 0.7 ThreadRng)  */
/* ======================================================================================== */
#define ORC_SEED_SALT 0x76616E52696A6E31ULL /* "vanRijn1" */
#define ORC_WEYL32 0x9E3779B9u            /* the draw counter's step */
#define ORC_LO_OFFSET 0x6A09E667u         /* the low word hashes the counter plus this */

uint64_t orc_mix64(uint64_t z) { /* splitmix64's finaliser */
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* Wellons' "lowbias32" 32-bit integer hash (two multiplies; a bijection) */
uint32_t orc_hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}

/* the per-(pixel, sample) stream base: one mix of the key and the (pixel, sample) pair as one 64-bit
 * word (injective for pixel, sample < 2^32), keyed by the seed */
uint64_t orc_stream_base(uint64_t seed, uint64_t pixel_index, uint64_t sample_index) {
    const uint64_t key = orc_mix64(seed ^ ORC_SEED_SALT);
    return orc_mix64(key ^ ((pixel_index << 32) + sample_index));
}

/* draw k (0-based): a 32-bit Weyl counter from the base's low word, xored with its high word, hashed
 * twice (high word: the counter, low word: the counter plus a constant) */
uint64_t orc_stream_draw(uint64_t base, uint64_t k) {
    const uint32_t x = (uint32_t)base + (uint32_t)(k + 1) * ORC_WEYL32;
    const uint32_t v = x ^ (uint32_t)(base >> 32);
    return ((uint64_t)orc_hash32(v) << 32) | orc_hash32(v + ORC_LO_OFFSET);
}

/* rand 0.7 `Standard` for f64: 53 high bits times 2^-53 (camera.rs:49, photon.rs:21) */
double orc_u64_to_standard(uint64_t u) { return (double)(u >> 11) * 0x1.0p-53; }

/* rand 0.7 `Open01` for f64: 52 bits into [1,2), minus (1 - EPSILON/2) (lambertian_material.rs:39-48) */
double orc_u64_to_open01(uint64_t u) {
    uint64_t bits = (u >> 12) | 0x3FF0000000000000ULL;
    double f;
    memcpy(&f, &bits, sizeof f);
    return f - (1.0 - 0x1.0p-53);
}

typedef struct orc_rng {
    uint64_t base;
    uint64_t k;
} orc_rng;

static double rng_standard(orc_rng* r) { return orc_u64_to_standard(orc_stream_draw(r->base, r->k++)); }
static double rng_open01(orc_rng* r) { return orc_u64_to_open01(orc_stream_draw(r->base, r->k++)); }
/* rand 0.7 Standard bool = (next_u32() as i32) < 0 with next_u32 = the draw's high half
 * (smooth_transparent_dialectric.rs:103) */
static int rng_bool(orc_rng* r) { return (int32_t)(uint32_t)(orc_stream_draw(r->base, r->k++) >> 32) < 0; }

/* ======================================================================================== */
/* Vec3 / Mat3 (src/math/vec3.rs, src/math/mat3.rs, src/math/mat2.rs)                     */
/* ======================================================================================== */
typedef struct v3 {
    double x, y, z;
} v3;

static v3 mk(double x, double y, double z) {
    v3 r = {x, y, z};
    return r;
}
static v3 ld(const double* p) { return mk(p[0], p[1], p[2]); }
static void st(double* p, v3 v) {
    p[0] = v.x;
    p[1] = v.y;
    p[2] = v.z;
}
static v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 scl(v3 a, double s) { return mk(a.x * s, a.y * s, a.z * s); }
static v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
static v3 vabs(v3 a) { return mk(fabs(a.x), fabs(a.y), fabs(a.z)); }
static double get(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

/* vec3.rs:76-82: zip-map-sum; `impl Sum for f64` folds from -0.0 (Rust >= 1.83) */
static double dot(v3 a, v3 b) {
    double s = -0.0;
    s = s + a.x * b.x;
    s = s + a.y * b.y;
    s = s + a.z * b.z;
    return s;
}
/* vec3.rs:84-89 */
static v3 cross(v3 a, v3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static double norm(v3 a) { return sqrt(dot(a, a)); }
/* vec3.rs:103-110: multiply by the reciprocal of the norm */
static v3 normalize(v3 a) {
    double inv = 1.0 / norm(a);
    return mk(a.x * inv, a.y * inv, a.z * inv);
}
void orc_normalize(const double v[3], double out[3]) { st(out, normalize(ld(v))); }

/* vec3.rs:112-127 */
static int smallest_coord(v3 v) {
    double x = fabs(v.x), y = fabs(v.y), z = fabs(v.z);
    if (x < y) return x < z ? 0 : 2;
    return y < z ? 1 : 2;
}

typedef struct m3 {
    double e[3][3];
} m3;

/* mat3.rs:34-42 */
static m3 from_rows(v3 r0, v3 r1, v3 r2) {
    m3 m;
    m.e[0][0] = r0.x; m.e[0][1] = r0.y; m.e[0][2] = r0.z;
    m.e[1][0] = r1.x; m.e[1][1] = r1.y; m.e[1][2] = r1.z;
    m.e[2][0] = r2.x; m.e[2][1] = r2.y; m.e[2][2] = r2.z;
    return m;
}
/* mat3.rs:72-90 + mat2.rs:13-15: determinant of the row-major remainder */
static double first_minor(const m3* m, int row, int col) {
    double el[2][2];
    int id = 0;
    for (int i = 0; i < 3; ++i) {
        if (i == row) continue;
        int jd = 0;
        for (int j = 0; j < 3; ++j) {
            if (j == col) continue;
            el[id][jd++] = m->e[i][j];
        }
        id++;
    }
    return el[0][0] * el[1][1] - el[0][1] * el[1][0];
}
/* mat3.rs:92-94: (-1)^(i+j) as f64 times the minor */
static double cofactor(const m3* m, int r, int c) { return (((r + c) & 1) ? -1.0 : 1.0) * first_minor(m, r, c); }
/* mat3.rs:106-109 */
static double determinant(const m3* m) {
    return m->e[0][0] * first_minor(m, 0, 0) - m->e[0][1] * first_minor(m, 0, 1) + m->e[0][2] * first_minor(m, 0, 2);
}
/* mat3.rs:111-118: cofactor_matrix().transpose() * determinant  (times, not divided by) */
static int try_inverse(const m3* m, m3* out) {
    double det = determinant(m);
    if (det == 0.0) return 0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) out->e[i][j] = cofactor(m, j, i) * det;
    return 1;
}
/* mat3.rs:147-157: row dots */
static v3 mul_mv(const m3* m, v3 v) {
    return mk(dot(mk(m->e[0][0], m->e[0][1], m->e[0][2]), v), dot(mk(m->e[1][0], m->e[1][1], m->e[1][2]), v),
              dot(mk(m->e[2][0], m->e[2][1], m->e[2][2]), v));
}
int orc_mat3_inverse(const double in[9], double out[9]) {
    m3 m, r;
    memcpy(m.e, in, sizeof m.e);
    if (!try_inverse(&m, &r)) return 0;
    memcpy(out, r.e, sizeof r.e);
    return 1;
}
double orc_mat3_determinant(const double in[9]) {
    m3 m;
    memcpy(m.e, in, sizeof m.e);
    return determinant(&m);
}
/* mat3.rs:72-90 (first_minor), :96-104 (cofactor_matrix), :62-70 (transpose), :121-132 (Mat3 *
 * Mat3: row(i) . column(j)), :147-157 (Mat3 * Vec3); exported for the reference's mat3 tests */
double orc_mat3_first_minor(const double in[9], int32_t row, int32_t column) {
    m3 m;
    memcpy(m.e, in, sizeof m.e);
    return first_minor(&m, row, column);
}
void orc_mat3_cofactor_matrix(const double in[9], double out[9]) {
    m3 m;
    memcpy(m.e, in, sizeof m.e);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) out[3 * i + j] = cofactor(&m, i, j);
}
void orc_mat3_transpose(const double in[9], double out[9]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) out[3 * i + j] = in[3 * j + i];
}
void orc_mat3_mul(const double a[9], const double b[9], double out[9]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            out[3 * i + j] = dot(mk(a[3 * i], a[3 * i + 1], a[3 * i + 2]), mk(b[j], b[3 + j], b[6 + j]));
}
void orc_mat3_mul_vec(const double in[9], const double v[3], double out[3]) {
    m3 m;
    memcpy(m.e, in, sizeof m.e);
    st(out, mul_mv(&m, ld(v)));
}
/* util/algebra_utils.rs:3-5: try_change_of_basis_matrix = Some(Mat3::from_rows(x, y, z)) */
void orc_change_of_basis(const double x[3], const double y[3], const double z[3], double out[9]) {
    m3 m = from_rows(ld(x), ld(y), ld(z));
    memcpy(out, m.e, sizeof m.e);
}

/* ======================================================================================== */
/* Interval / BoundingBox (src/util/interval.rs, src/util/axis_aligned_bounding_box.rs)     */
/* ======================================================================================== */
/* Rust f64::max / f64::min ignore a NaN operand: C fmax / fmin */
typedef struct ival {
    double min, max;
} ival;
static ival ival_new(double a, double b) { /* interval.rs:8-14 */
    ival r;
    if (a > b) { r.min = b; r.max = a; } else { r.min = a; r.max = b; }
    return r;
}
static ival ival_empty(void) { ival r = {INFINITY, -INFINITY}; return r; }
static int ival_is_empty(ival a) { return a.min > a.max; }
static int ival_is_degenerate(ival a) { return a.min == a.max; }
static ival ival_union(ival a, ival b) { /* interval.rs:66-77 */
    if (ival_is_empty(a)) return b;
    if (ival_is_empty(b)) return a;
    ival r = {fmin(a.min, b.min), fmax(a.max, b.max)};
    return r;
}
static ival ival_expand(ival a, double v) { /* interval.rs:79-87 */
    if (ival_is_empty(a)) { ival r = {v, v}; return r; }
    ival r = {fmin(a.min, v), fmax(a.max, v)};
    return r;
}

typedef struct bbox {
    ival b[3];
} bbox;
static bbox bbox_empty(void) { bbox r = {{ival_empty(), ival_empty(), ival_empty()}}; return r; }
static bbox bbox_union(bbox a, bbox b) {
    bbox r;
    for (int i = 0; i < 3; ++i) r.b[i] = ival_union(a.b[i], b.b[i]);
    return r;
}
static bbox bbox_expand(bbox a, v3 p) {
    a.b[0] = ival_expand(a.b[0], p.x);
    a.b[1] = ival_expand(a.b[1], p.y);
    a.b[2] = ival_expand(a.b[2], p.z);
    return a;
}
/* axis_aligned_bounding_box.rs:76-99 (util) */
static int largest_dimension(bbox bb) {
    int acc = 0;
    double acc_size = 0.0;
    for (int i = 0; i < 3; ++i) {
        double size = ival_is_degenerate(bb.b[i]) ? -1.0 : bb.b[i].max - bb.b[i].min;
        if (size > acc_size) { acc = i; acc_size = size; }
    }
    return acc;
}

/* raycasting/axis_aligned_bounding_box.rs:9-27: line (not ray) slab test; also reports the
 * final interval so pruned mode can cull by distance */
static int slab(const bbox* bb, v3 o, v3 d, double* tlo, double* thi) {
    double lo = -INFINITY, hi = INFINITY;
    double oc[3] = {o.x, o.y, o.z}, dc[3] = {d.x, d.y, d.z};
    for (int i = 0; i < 3; ++i) {
        ival t = ival_new((bb->b[i].min - oc[i]) / dc[i], (bb->b[i].max - oc[i]) / dc[i]);
        lo = fmax(lo, t.min);
        hi = fmin(hi, t.max);
        if (lo > hi) return 0;
    }
    *tlo = lo;
    *thi = hi;
    return 1;
}
int orc_bbox_intersect(const double bmin[3], const double bmax[3], const double o[3], const double d[3]) {
    bbox bb; /* BoundingBox::from_corners (util/axis_aligned_bounding_box.rs:11-21) */
    for (int i = 0; i < 3; ++i) bb.b[i] = ival_new(bmin[i], bmax[i]);
    double a, b;
    return slab(&bb, ld(o), ld(d), &a, &b);
}

/* Interval (util/interval.rs:7-87) and util BoundingBox (util/axis_aligned_bounding_box.rs:11-99)
 * exported as {min, max} pairs / six doubles {min x, max x, min y, max y, min z, max z}, for the
 * reference's interval and bbox tests.  contains_value: interval.rs:53-55. */
static ival ival_ld(const double a[2]) { ival r = {a[0], a[1]}; return r; }
static void ival_st(double out[2], ival a) { out[0] = a.min; out[1] = a.max; }
void orc_interval_new(double a, double b, double out[2]) { ival_st(out, ival_new(a, b)); }
void orc_interval_union(const double a[2], const double b[2], double out[2]) {
    ival_st(out, ival_union(ival_ld(a), ival_ld(b)));
}
void orc_interval_intersection(const double a[2], const double b[2], double out[2]) { /* interval.rs:57-62 */
    ival r = {fmax(a[0], b[0]), fmin(a[1], b[1])};
    ival_st(out, r);
}
void orc_interval_expand(const double a[2], double v, double out[2]) { ival_st(out, ival_expand(ival_ld(a), v)); }
int orc_interval_is_empty(const double a[2]) { return ival_is_empty(ival_ld(a)); }
int orc_interval_is_degenerate(const double a[2]) { return ival_is_degenerate(ival_ld(a)); }
int orc_interval_contains(const double a[2], double v) { return v >= a[0] && v <= a[1]; }

static bbox bbox_ld(const double b[6]) {
    bbox r;
    for (int i = 0; i < 3; ++i) { r.b[i].min = b[2 * i]; r.b[i].max = b[2 * i + 1]; }
    return r;
}
static void bbox_st(double out[6], bbox b) {
    for (int i = 0; i < 3; ++i) { out[2 * i] = b.b[i].min; out[2 * i + 1] = b.b[i].max; }
}
void orc_bbox_from_corners(const double a[3], const double b[3], double out[6]) { /* :11-21 */
    bbox r;
    for (int i = 0; i < 3; ++i) r.b[i] = ival_new(a[i], b[i]);
    bbox_st(out, r);
}
void orc_bbox_from_points(int64_t n, const double* pts, double out[6]) { /* :40-47 fold expand_to_point */
    bbox r = bbox_empty();
    for (int64_t k = 0; k < n; ++k) r = bbox_expand(r, ld(pts + 3 * k));
    bbox_st(out, r);
}
void orc_bbox_union(const double a[6], const double b[6], double out[6]) { bbox_st(out, bbox_union(bbox_ld(a), bbox_ld(b))); }
int orc_bbox_contains_point(const double b[6], const double p[3]) { /* :59-64 */
    for (int i = 0; i < 3; ++i)
        if (!(p[i] >= b[2 * i] && p[i] <= b[2 * i + 1])) return 0;
    return 1;
}
int orc_bbox_largest_dimension(const double b[6]) { return largest_dimension(bbox_ld(b)); }

/* ======================================================================================== */
/* Ray (src/raycasting/mod.rs:29-61)                                                        */
/* ======================================================================================== */
typedef struct ray {
    v3 o, d;
} ray;
static ray ray_new(v3 o, v3 d) { ray r = {o, normalize(d)}; return r; }
static v3 point_at(const ray* r, double t) { return add(r->o, scl(r->d, t)); }
static ray ray_bias(const ray* r, double a) { return ray_new(point_at(r, a), r->d); }
/* Ray::new / point_at (mod.rs:41-52), exported for the reference's ray tests (mod.rs:155-181) */
void orc_ray_new(const double o[3], const double d[3], double out_o[3], double out_d[3]) {
    ray r = ray_new(ld(o), ld(d));
    st(out_o, r.o);
    st(out_d, r.d);
}
void orc_ray_point_at(const double o[3], const double d[3], double t, double out[3]) {
    ray r = {ld(o), ld(d)};
    st(out, point_at(&r, t));
}

/* ======================================================================================== */
/* Primitives                                                                               */
/* ======================================================================================== */
static void hit_clear(orc_hit* h) { memset(h, 0, sizeof *h); }

/* triangle.rs:108-122: NOTE compares signed components, not magnitudes */
static void perm_indices(v3 v, int idx[3]) {
    if (v.x > v.y) {
        if (v.z > v.x) { idx[0] = 0; idx[1] = 1; idx[2] = 2; }
        else { idx[0] = 1; idx[1] = 2; idx[2] = 0; }
    } else {
        if (v.z > v.y) { idx[0] = 0; idx[1] = 1; idx[2] = 2; }
        else { idx[0] = 2; idx[1] = 0; idx[2] = 1; }
    }
}
static v3 permute(v3 v, const int idx[3]) { return mk(get(v, idx[0]), get(v, idx[1]), get(v, idx[2])); }

/* triangle.rs:35-98 (+ helpers :108-162).  Decision part and shading part. */
static void triangle_intersect(const double* vv, const double* nn, const ray* r, orc_hit* out) {
    hit_clear(out);
    v3 V[3] = {ld(vv), ld(vv + 3), ld(vv + 6)};
    v3 translation = neg(r->o);
    int idx[3];
    perm_indices(r->d, idx);
    v3 pd = permute(r->d, idx);
    double sx = -pd.x / pd.z, sy = -pd.y / pd.z; /* calculate_shear_to_z_axis :129-131 */
    v3 T[3];
    for (int i = 0; i < 3; ++i) {
        v3 p = permute(add(V[i], translation), idx);
        T[i] = mk(p.x + sx * p.z, p.y + sy * p.z, p.z); /* apply_shear_to_z_axis :133-135 */
    }
    /* signed_edge_functions :141-158: e0=E(v1,v2), e1=E(v2,v0), e2=E(v0,v1) */
    double e0 = T[1].x * T[2].y - T[2].x * T[1].y;
    double e1 = T[2].x * T[0].y - T[0].x * T[2].y;
    double e2 = T[0].x * T[1].y - T[1].x * T[0].y;
    int allpos = !signbit(e0) && !signbit(e1) && !signbit(e2);
    int allneg = signbit(e0) && signbit(e1) && signbit(e2);
    if (!(allpos || allneg)) return;
    /* barycentric_coordinates_from_signed_edge_functions :160-162, fold from 0.0 */
    v3 ea = vabs(mk(e0, e1, e2));
    double s = 0.0;
    s = s + ea.x;
    s = s + ea.y;
    s = s + ea.z;
    double inv = 1.0 / s;
    v3 b = mk(ea.x * inv, ea.y * inv, ea.z * inv);
    double tz = 0.0; /* :57-61, explicit fold(0.0) */
    tz = tz + T[0].z * b.x;
    tz = tz + T[1].z * b.y;
    tz = tz + T[2].z * b.z;
    if ((!signbit(tz)) != (!signbit(pd.z))) return;
    v3 loc = mk(0.0, 0.0, 0.0); /* :66-71, fold(Vec3::zeros()) */
    loc = add(loc, scl(V[0], b.x));
    loc = add(loc, scl(V[1], b.y));
    loc = add(loc, scl(V[2], b.z));
    out->valid = 1;
    out->distance = norm(sub(r->o, loc));
    st(out->location, loc);
    if (nn) {
        v3 N[3] = {ld(nn), ld(nn + 3), ld(nn + 6)};
        v3 nsum = mk(0.0, 0.0, 0.0);
        nsum = add(nsum, scl(N[0], b.x));
        nsum = add(nsum, scl(N[1], b.y));
        nsum = add(nsum, scl(N[2], b.z));
        v3 n = normalize(nsum);
        v3 cot = normalize(cross(sub(V[0], V[1]), n));
        v3 tan = normalize(cross(cot, n));
        st(out->normal, n);
        st(out->cotangent, cot);
        st(out->tangent, tan);
        st(out->retro, normalize(sub(r->o, loc)));
    }
}
void orc_triangle_intersect(const double v[9], const double n[9], const double o[3], const double d[3], orc_hit* out) {
    ray r = {ld(o), ld(d)};
    triangle_intersect(v, n, &r, out);
}

/* sphere.rs:39-93 */
static void sphere_intersect(v3 c, double radius, const ray* r, orc_hit* out) {
    hit_clear(out);
    v3 o = r->o, d = r->d;
    double a = 0.0;
    a = a + d.x * d.x;
    a = a + d.y * d.y;
    a = a + d.z * d.z;
    v3 bv = scl(sub(mk(o.x * d.x, o.y * d.y, o.z * d.z), mk(c.x * d.x, c.y * d.y, c.z * d.z)), 2.0);
    double b = 0.0;
    b = b + bv.x;
    b = b + bv.y;
    b = b + bv.z;
    v3 cv = sub(add(mk(o.x * o.x, o.y * o.y, o.z * o.z), mk(c.x * c.x, c.y * c.y, c.z * c.z)),
                scl(mk(c.x * o.x, c.y * o.y, c.z * o.z), 2.0));
    double cc = 0.0;
    cc = cc + cv.x;
    cc = cc + cv.y;
    cc = cc + cv.z;
    cc = cc - radius * radius;
    double delta_squared = b * b - 4.0 * a * cc;
    if (delta_squared < 0.0) return;
    double delta = sqrt(delta_squared);
    double one_over_2_a = 1.0 / (2.0 * a);
    double t1 = (-b - delta) * one_over_2_a;
    double t2 = (-b + delta) * one_over_2_a;
    double distance = (t1 < 0.0 || (t2 >= 0.0 && t1 >= t2)) ? t2 : t1;
    if (distance <= 0.0) return;
    v3 loc = point_at(r, distance);
    v3 n = normalize(sub(loc, c));
    v3 tan = normalize(cross(n, mk(0.0, 0.0, 1.0)));
    v3 cot = cross(n, tan);
    out->valid = 1;
    out->distance = distance;
    st(out->location, loc);
    st(out->normal, n);
    st(out->tangent, tan);
    st(out->cotangent, cot);
    st(out->retro, neg(d));
}
void orc_sphere_intersect(const double centre[3], double radius, const double o[3], const double d[3], orc_hit* out) {
    ray r = {ld(o), ld(d)};
    sphere_intersect(ld(centre), radius, &r, out);
}

/* plane.rs:18-31 */
void orc_plane_new(const double normal_in[3], double on[3], double ot[3], double oc[3]) {
    v3 n = normalize(ld(normal_in));
    v3 axis = mk(0.0, 0.0, 0.0);
    int k = smallest_coord(n);
    if (k == 0) axis.x = 1.0; else if (k == 1) axis.y = 1.0; else axis.z = 1.0;
    v3 cot = normalize(cross(n, axis));
    v3 tan = cross(n, cot);
    st(on, n);
    st(ot, tan);
    st(oc, cot);
}
/* plane.rs:49-75 */
static void plane_intersect(v3 n, v3 tan, v3 cot, double dist, const ray* r, orc_hit* out) {
    hit_clear(out);
    double dn = dot(r->d, n);
    v3 p = scl(n, dist);
    double num = dot(sub(p, r->o), n);
    if (dn == 0.0) {
        if (num != 0.0) return;
    }
    double t = num / dn;
    if (t < 0.0) return;
    out->valid = 1;
    out->distance = t;
    st(out->location, point_at(r, t));
    st(out->normal, n);
    st(out->tangent, tan);
    st(out->cotangent, cot);
    st(out->retro, neg(r->d));
}
void orc_plane_intersect(const double n[3], const double t[3], const double c[3], double dist, const double o[3],
                         const double d[3], orc_hit* out) {
    ray r = {ld(o), ld(d)};
    plane_intersect(ld(n), ld(t), ld(c), dist, &r, out);
}

/* ======================================================================================== */
/* Spectrum / colour (src/colour/spectrum.rs, colour_xyz.rs, photon.rs, mod.rs:13-14)       */
/* ======================================================================================== */
#define SHORTEST_VISIBLE 380.0
#define LONGEST_VISIBLE 740.0

/* spectrum.rs:50-79 */
double orc_spectrum_intensity(double shortest, double longest, int32_t n, const double* s, double wl) {
    if (wl < shortest || wl > longest) return 0.0;
    double range = longest - shortest;
    size_t i = (size_t)((double)(n - 1) * ((wl - shortest) / range));
    double before = (double)i / (double)(n - 1) * range + shortest;
    if (i == (size_t)(n - 1)) return s[i];
    double after = (double)(i + 1) / (double)(n - 1) * range + shortest;
    double delta = after - before;
    double ratio = (wl - before) / delta;
    return s[i] * (1.0 - ratio) + s[i + 1] * ratio;
}

/* spectrum.rs:81-165: Smits-style basis selection on the channel order */
void orc_reflection_from_linear_rgb(double r, double g, double b, double out[32]) {
    const double* W = orc_rgbspec_basis[ORC_RGBSPEC_WHITE];
    int kx, ky;
    double c0, c1, c2;
    if (r <= g && r <= b) {
        if (g <= b) { c0 = r; c1 = g - r; c2 = b - g; kx = ORC_RGBSPEC_CYAN; ky = ORC_RGBSPEC_BLUE; }
        else { c0 = r; c1 = b - r; c2 = g - b; kx = ORC_RGBSPEC_CYAN; ky = ORC_RGBSPEC_GREEN; }
    } else if (g <= r && g < b) {
        if (r <= b) { c0 = g; c1 = r - g; c2 = b - r; kx = ORC_RGBSPEC_MAGENTA; ky = ORC_RGBSPEC_BLUE; }
        else { c0 = g; c1 = b - g; c2 = r - b; kx = ORC_RGBSPEC_MAGENTA; ky = ORC_RGBSPEC_RED; }
    } else {
        if (r <= g) { c0 = b; c1 = r - b; c2 = g - r; kx = ORC_RGBSPEC_YELLOW; ky = ORC_RGBSPEC_GREEN; }
        else { c0 = b; c1 = g - b; c2 = r - g; kx = ORC_RGBSPEC_YELLOW; ky = ORC_RGBSPEC_RED; }
    }
    const double* X = orc_rgbspec_basis[kx];
    const double* Y = orc_rgbspec_basis[ky];
    for (int i = 0; i < 32; ++i) out[i] = c0 * W[i] + c1 * X[i] + c2 * Y[i];
}

/* colour_xyz.rs:86-89: alpha * exp(-(t^2) / (2 sigma^2)), sigma by side of mu; powi(2) = x*x */
static double gaussian(double wl, double alpha, double mu, double s1, double s2) {
    double s = wl < mu ? s1 : s2;
    double denominator = 2.0 * (s * s);
    double t = wl - mu;
    return alpha * exp(-(t * t) / denominator);
}
/* colour_xyz.rs:91-103 */
void orc_colour_xyz_for_wavelength(double wl, double out[3]) {
    out[0] = gaussian(wl, 1.056, 599.8, 37.9, 31.0) + gaussian(wl, 0.362, 442.0, 16.0, 26.7) +
             gaussian(wl, -0.065, 501.1, 20.4, 26.2);
    out[1] = gaussian(wl, 0.821, 568.8, 46.9, 40.5) + gaussian(wl, 0.286, 530.9, 16.3, 31.1);
    out[2] = gaussian(wl, 1.217, 437.0, 11.8, 36.0) + gaussian(wl, 0.681, 459.0, 26.0, 13.8);
}
/* colour_xyz.rs:49-67 */
void orc_colour_xyz_to_linear_rgb(const double xyz[3], double rgb[3]) {
    m3 t = from_rows(mk(3.24096994, -1.53738318, -0.49861076), mk(-0.96924364, 1.87596750, 0.04155506),
                     mk(0.05563008, -0.20397696, 1.05697151));
    st(rgb, mul_mv(&t, ld(xyz)));
}
void orc_colour_xyz_from_linear_rgb(const double rgb[3], double xyz[3]) {
    m3 t = from_rows(mk(0.41239080, 0.35758434, 0.18048079), mk(0.21263901, 0.71516868, 0.07219232),
                     mk(0.01933082, 0.11919478, 0.95053215));
    st(xyz, mul_mv(&t, ld(rgb)));
}

/* colour_xyz.rs:78-84: srgb_gamma with the reference's constants (12.98, 1.005) */
static double srgb_gamma(double u) {
    if (u <= 0.0031308) return 12.98 * u;
    return 1.005 * pow(u, 1.0 / 2.4) - 0.055;
}
/* image.rs:110-128,141-145: f64::clamp(0, 1) keeps NaN; Rust's `as u8` saturates, NaN -> 0 */
static uint8_t clamp_to_byte(double v) {
    if (v != v) return 0;
    double c = v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v);
    return (uint8_t)(c * 255.0);
}
/* ClampingToneMapper for ColourXyz (image.rs:166-187) over ColourXyz::to_srgb
 * (colour_xyz.rs:69-76): colour buffer [n][3] -> RGB bytes [n][3] */
void orc_tone_map(const double* colour, uint64_t n, uint8_t* rgb) {
    for (uint64_t i = 0; i < n; ++i) {
        double lin[3];
        orc_colour_xyz_to_linear_rgb(colour + 3 * i, lin);
        for (int k = 0; k < 3; ++k) rgb[3 * i + k] = clamp_to_byte(srgb_gamma(lin[k]));
    }
}

/* simple_random_integrator.rs:57-65: sky = reflection_from_linear_rgb((w.y, w.y, 1)) at lambda */
double orc_sky_intensity(const double w[3], double wl) {
    double s[32];
    orc_reflection_from_linear_rgb(w[1], w[1], 1.0, s);
    return orc_spectrum_intensity(ORC_RGBSPEC_SHORTEST, ORC_RGBSPEC_LONGEST, 32, s, wl);
}

/* ======================================================================================== */
/* Camera (src/camera.rs:13-67)                                                             */
/* ======================================================================================== */
static double cam_scale(uint64_t i, uint64_t n, double l, double u) {
    double nn = (double)n;
    double ii = (double)i;
    double pixel_size = l * (1.0 / nn);
    return (ii + u) * pixel_size;
}
void orc_ray_for_pixel(const double cam[3], uint64_t width, uint64_t height, uint64_t row, uint64_t column, double ux,
                       double uy, double o[3], double d[3]) {
    double w = (double)width, h = (double)height, fw, fh;
    if (w > h) { fw = w / h; fh = 1.0; } else { fw = 1.0; fh = w / h; } /* camera.rs:25-34 */
    double x = cam_scale(column, width, fw, ux) - fw * 0.5;
    double y = cam_scale(height - (row + 1), height, fh, uy) - fh * 0.5;
    ray r = ray_new(ld(cam), mk(x, y, 1.0));
    st(o, r.o);
    st(d, r.d);
}

/* ======================================================================================== */
/* Accumulation buffer (src/accumulation_buffer.rs:44-85)                                   */
/* ======================================================================================== */
void orc_update_pixel(double colour[3], double sum[3], double bias[3], double* weight, double* weight_bias, double wl,
                      double intensity, double w) {
    double c[3];
    orc_colour_xyz_for_wavelength(wl, c);
    for (int k = 0; k < 3; ++k) c[k] = c[k] * intensity; /* ColourXyz::from_photon */
    double wy = w - *weight_bias;
    double wt = *weight + wy;
    *weight_bias = (wt - *weight) - wy;
    *weight = wt;
    for (int k = 0; k < 3; ++k) {
        double y = c[k] * w - bias[k];
        double t = sum[k] + y;
        bias[k] = (t - sum[k]) - y;
        sum[k] = t;
    }
    double inv = 1.0 / *weight;
    for (int k = 0; k < 3; ++k) colour[k] = sum[k] * inv;
}

void orc_merge_tile(uint64_t dst_width, double* dst_colour, double* dst_weight, uint64_t start_row, uint64_t start_col,
                    uint64_t th, uint64_t tw, const double* src_colour, const double* src_weight) {
    for (uint64_t i = 0; i < th; ++i)
        for (uint64_t j = 0; j < tw; ++j) {
            uint64_t di = (start_row + i) * dst_width + (start_col + j), si = i * tw + j;
            double w1 = dst_weight[di], w2 = src_weight[si];
            double inv = 1.0 / (w1 + w2);
            for (int k = 0; k < 3; ++k)
                dst_colour[3 * di + k] = (dst_colour[3 * di + k] * w1 + src_colour[3 * si + k] * w2) * inv;
            dst_weight[di] = dst_weight[di] + w2;
        }
}

/* ======================================================================================== */
/* Scene                                                                                    */
/* ======================================================================================== */
typedef struct orc_material {
    int kind;
    double shortest, longest;
    int n;
    double s[64];
    double diffuse, reflection; /* reflection = Phong's specular_strength */
    double smoothness;          /* Phong */
} orc_material;

typedef struct orc_prim {
    int kind, material;
    v3 vec, tan, cot; /* plane: normal/tangent/cotangent (Plane::new); sphere: centre */
    double scalar;
} orc_prim;

/* BVH node: reference enum BoundingVolumeHierarchy (bounding_volume_hierarchy.rs:18-28) */
typedef struct bvh_node {
    bbox bounds;
    int64_t left, right; /* node indices; -1 for a leaf */
    int64_t first, count; /* leaf: range in the leaf-ordered primitive array */
} bvh_node;

typedef struct orc_object {
    int kind; /* 0 primitive list, 1 mesh BVH */
    int prim_first, prim_count;
    /* mesh */
    int64_t ntri;
    double* verts;   /* leaf order, 9 per triangle */
    double* norms;   /* leaf order */
    int64_t* orig;   /* leaf order -> input triangle index */
    bvh_node* nodes;
    int64_t nnodes;
    int depth;
    int material;
} orc_object;

struct orc_scene {
    v3 camera;
    /* WhittedIntegrator (whitted_integrator.rs:15-87) when whitted != 0 */
    int whitted;
    orc_material ambient;
    int nlights;
    v3 light_dir[16];
    orc_material light[16];
    orc_material* mats;
    int nmats;
    orc_prim* prims;
    int nprims;
    orc_object* objs;
    int nobjs;
    double extent; /* max |coordinate| over camera and geometry: scales the pruned-mode margins */
};

orc_scene* orc_scene_new(const double camera[3]) {
    orc_scene* s = (orc_scene*)calloc(1, sizeof *s);
    s->camera = ld(camera);
    s->extent = fmax(fmax(fabs(camera[0]), fabs(camera[1])), fabs(camera[2]));
    return s;
}
void orc_scene_free(orc_scene* s) {
    if (!s) return;
    for (int i = 0; i < s->nobjs; ++i) {
        free(s->objs[i].verts);
        free(s->objs[i].norms);
        free(s->objs[i].orig);
        free(s->objs[i].nodes);
    }
    free(s->objs);
    free(s->prims);
    free(s->mats);
    free(s);
}
int orc_scene_add_material(orc_scene* s, int32_t kind, double shortest, double longest, int32_t n,
                           const double* samples, double diffuse, double reflection, double smoothness) {
    if (n < 1 || n > 64) return -1;
    s->mats = (orc_material*)realloc(s->mats, sizeof(orc_material) * (s->nmats + 1));
    orc_material* m = &s->mats[s->nmats];
    memset(m, 0, sizeof *m);
    m->kind = kind;
    m->shortest = shortest;
    m->longest = longest;
    m->n = n;
    memcpy(m->s, samples, sizeof(double) * n);
    m->diffuse = diffuse;
    m->reflection = reflection;
    m->smoothness = smoothness;
    return s->nmats++;
}
static void grow_objs(orc_scene* s) { s->objs = (orc_object*)realloc(s->objs, sizeof(orc_object) * (s->nobjs + 1)); }

int orc_scene_add_primitive_list(orc_scene* s, int32_t count, const int32_t* kinds, const int32_t* mats,
                                 const double* vecs, const double* scalars) {
    grow_objs(s);
    orc_object* o = &s->objs[s->nobjs];
    memset(o, 0, sizeof *o);
    o->kind = 0;
    o->prim_first = s->nprims;
    o->prim_count = count;
    s->prims = (orc_prim*)realloc(s->prims, sizeof(orc_prim) * (s->nprims + count));
    for (int i = 0; i < count; ++i) {
        orc_prim* p = &s->prims[s->nprims + i];
        memset(p, 0, sizeof *p);
        p->kind = kinds[i];
        p->material = mats[i];
        p->scalar = scalars[i];
        if (kinds[i] == ORC_PRIM_PLANE) {
            double n[3], t[3], c[3];
            orc_plane_new(vecs + 3 * i, n, t, c);
            p->vec = ld(n);
            p->tan = ld(t);
            p->cot = ld(c);
            s->extent = fmax(s->extent, fabs(scalars[i]));
        } else {
            p->vec = ld(vecs + 3 * i);
            for (int k = 0; k < 3; ++k) s->extent = fmax(s->extent, fabs(vecs[3 * i + k]) + fabs(scalars[i]));
        }
    }
    s->nprims += count;
    return s->nobjs++;
}

/* ---- BVH build: bounding_volume_hierarchy.rs:30-74 ---- */
typedef struct build_prim {
    bbox bb;
    double centre[3];
    int64_t orig;
} build_prim;

static int g_sort_axis; /* build is single threaded */
/* sort_unstable_by(centre[axis].partial_cmp) with NaN -> Equal; ties broken by input index so the
 * permutation is unique (pdqsort's order of equal keys is implementation-defined; the product
 * uses the same tie rule) */
static int cmp_centre(const void* a, const void* b) {
    const build_prim* x = (const build_prim*)a;
    const build_prim* y = (const build_prim*)b;
    double cx = x->centre[g_sort_axis], cy = y->centre[g_sort_axis];
    if (cx < cy) return -1;
    if (cx > cy) return 1;
    return (x->orig > y->orig) - (x->orig < y->orig);
}

typedef struct builder {
    build_prim* p;
    bvh_node* nodes;
    int64_t nnodes, cap;
    int depth;
} builder;

static int64_t build_rec(builder* B, int64_t lo, int64_t hi, int level) {
    if (level + 1 > B->depth) B->depth = level + 1;
    bbox bounds = bbox_empty();
    for (int64_t i = lo; i < hi; ++i) bounds = bbox_union(bounds, B->p[i].bb);
    if (B->nnodes == B->cap) {
        B->cap = B->cap ? 2 * B->cap : 1024;
        B->nodes = (bvh_node*)realloc(B->nodes, sizeof(bvh_node) * B->cap);
    }
    int64_t me = B->nnodes++;
    B->nodes[me].bounds = bounds;
    if (hi - lo <= 1) {
        B->nodes[me].left = B->nodes[me].right = -1;
        B->nodes[me].first = lo;
        B->nodes[me].count = hi - lo;
        return me;
    }
    g_sort_axis = largest_dimension(bounds);
    qsort(B->p + lo, (size_t)(hi - lo), sizeof(build_prim), cmp_centre);
    int64_t pivot = (hi - lo) / 2;
    int64_t l = build_rec(B, lo, lo + pivot, level + 1);
    int64_t r = build_rec(B, lo + pivot, hi, level + 1);
    B->nodes[me].left = l;
    B->nodes[me].right = r;
    B->nodes[me].first = 0;
    B->nodes[me].count = 0;
    return me;
}

int orc_scene_add_mesh(orc_scene* s, int64_t ntri, const double* verts, const double* norms, int32_t material) {
    grow_objs(s);
    orc_object* o = &s->objs[s->nobjs];
    memset(o, 0, sizeof *o);
    o->kind = 1;
    o->material = material;
    o->ntri = ntri;
    builder B = {0};
    B.p = (build_prim*)malloc(sizeof(build_prim) * (size_t)(ntri ? ntri : 1));
    for (int64_t t = 0; t < ntri; ++t) {
        bbox bb = bbox_empty(); /* BoundingBox::from_points(&self.vertices) (triangle.rs:101-105) */
        for (int k = 0; k < 3; ++k) {
            bb = bbox_expand(bb, ld(verts + 9 * t + 3 * k));
            for (int c = 0; c < 3; ++c) s->extent = fmax(s->extent, fabs(verts[9 * t + 3 * k + c]));
        }
        B.p[t].bb = bb;
        for (int c = 0; c < 3; ++c) B.p[t].centre[c] = (bb.b[c].min + bb.b[c].max) / 2.0; /* centre() :30-36 */
        B.p[t].orig = t;
    }
    build_rec(&B, 0, ntri, 0);
    o->nodes = B.nodes;
    o->nnodes = B.nnodes;
    o->depth = B.depth;
    o->verts = (double*)malloc(sizeof(double) * 9 * (size_t)(ntri ? ntri : 1));
    o->norms = (double*)malloc(sizeof(double) * 9 * (size_t)(ntri ? ntri : 1));
    o->orig = (int64_t*)malloc(sizeof(int64_t) * (size_t)(ntri ? ntri : 1));
    for (int64_t i = 0; i < ntri; ++i) {
        int64_t t = B.p[i].orig;
        o->orig[i] = t;
        memcpy(o->verts + 9 * i, verts + 9 * t, 9 * sizeof(double));
        memcpy(o->norms + 9 * i, norms + 9 * t, 9 * sizeof(double));
    }
    free(B.p);
    return s->nobjs++;
}

int orc_scene_mesh_leaf_order(const orc_scene* s, int32_t object, int64_t* out) {
    if (object < 0 || object >= s->nobjs || s->objs[object].kind != 1) return -1;
    memcpy(out, s->objs[object].orig, sizeof(int64_t) * (size_t)s->objs[object].ntri);
    return 0;
}
int orc_scene_mesh_depth(const orc_scene* s, int32_t object) {
    if (object < 0 || object >= s->nobjs || s->objs[object].kind != 1) return -1;
    return s->objs[object].depth;
}

/* ======================================================================================== */
/* Closest hit                                                                              */
/* ======================================================================================== */
typedef struct trace_ctx {
    orc_counters* cnt;
    int mode;
    double margin, behind_margin;
} trace_ctx;

/* bounding_volume_hierarchy.rs:77-92: on a tie the right (later) argument wins */
static void closest_of(orc_hit* a, const orc_hit* b) {
    if (!b->valid) return;
    if (!a->valid) { *a = *b; return; }
    if (a->distance < b->distance) return;
    *a = *b;
}

/* reference mode: bounding_volume_hierarchy.rs:94-120 (both children whenever the line crosses) */
static void bvh_ref(const orc_object* ob, int64_t node, const ray* r, trace_ctx* cx, orc_hit* out) {
    hit_clear(out);
    const bvh_node* nd = &ob->nodes[node];
    double lo, hi;
    cx->cnt->box_tests++;
    if (!slab(&nd->bounds, r->o, r->d, &lo, &hi)) return;
    if (nd->left < 0) {
        for (int64_t i = nd->first; i < nd->first + nd->count; ++i) {
            orc_hit h;
            cx->cnt->triangle_tests++;
            triangle_intersect(ob->verts + 9 * i, ob->norms + 9 * i, r, &h);
            if (h.valid) { h.primitive = i; h.material = ob->material; }
            closest_of(out, &h);
        }
        return;
    }
    orc_hit a, b;
    bvh_ref(ob, nd->left, r, cx, &a);
    bvh_ref(ob, nd->right, r, cx, &b);
    closest_of(&a, &b);
    *out = a;
}

/* pruned mode: same winner (closest distance, ties -> later in-order leaf), subtrees culled when
 * their line interval starts beyond the best distance (+margin) or ends behind the origin
 * (-margin, only when the ray's shear axis is not near zero).  Shading fields are filled for the
 * winner only. */
typedef struct pruned_best {
    double d;
    int64_t leaf;
    double bound; /* distance bound from earlier objects */
} pruned_best;

static void bvh_pruned(const orc_object* ob, int64_t node, const ray* r, trace_ctx* cx, int behind_ok, pruned_best* pb) {
    const bvh_node* nd = &ob->nodes[node];
    double lo, hi;
    cx->cnt->box_tests++;
    if (!slab(&nd->bounds, r->o, r->d, &lo, &hi)) return;
    double bound = fmin(pb->d, pb->bound);
    if (lo > bound + cx->margin * (1.0 + fabs(bound))) return;
    if (behind_ok && hi < -cx->behind_margin) return;
    if (nd->left < 0) {
        for (int64_t i = nd->first; i < nd->first + nd->count; ++i) {
            orc_hit h;
            cx->cnt->triangle_tests++;
            triangle_intersect(ob->verts + 9 * i, NULL, r, &h);
            if (!h.valid) continue;
            if (pb->leaf < 0 || h.distance < pb->d || (h.distance == pb->d && i > pb->leaf)) {
                pb->d = h.distance;
                pb->leaf = i;
            }
        }
        return;
    }
    /* near child first; visiting order does not change the winner */
    const bvh_node* L = &ob->nodes[nd->left];
    const bvh_node* R = &ob->nodes[nd->right];
    double l0, l1, r0, r1;
    int hl = slab(&L->bounds, r->o, r->d, &l0, &l1);
    int hr = slab(&R->bounds, r->o, r->d, &r0, &r1);
    (void)hl;
    (void)hr;
    if (hl && hr && r0 < l0) {
        bvh_pruned(ob, nd->right, r, cx, behind_ok, pb);
        bvh_pruned(ob, nd->left, r, cx, behind_ok, pb);
    } else {
        bvh_pruned(ob, nd->left, r, cx, behind_ok, pb);
        bvh_pruned(ob, nd->right, r, cx, behind_ok, pb);
    }
}

/* vec_aggregate.rs:11-22: min_by over the hits; on ties the FIRST stays (cmp::min_by) */
static void prim_list(const orc_scene* s, const orc_object* ob, const ray* r, orc_hit* out) {
    hit_clear(out);
    for (int i = 0; i < ob->prim_count; ++i) {
        const orc_prim* p = &s->prims[ob->prim_first + i];
        orc_hit h;
        if (p->kind == ORC_PRIM_PLANE) plane_intersect(p->vec, p->tan, p->cot, p->scalar, r, &h);
        else sphere_intersect(p->vec, p->scalar, r, &h);
        if (!h.valid) continue;
        h.primitive = i;
        h.material = p->material;
        if (!out->valid || out->distance > h.distance) *out = h;
    }
}

/* sampler.rs:9-20 */
static void sample_scene(const orc_scene* s, const ray* r, trace_ctx* cx, orc_hit* best) {
    hit_clear(best);
    cx->cnt->rays++;
    for (int oi = 0; oi < s->nobjs; ++oi) {
        const orc_object* ob = &s->objs[oi];
        orc_hit h;
        if (ob->kind == 0) {
            prim_list(s, ob, r, &h);
        } else if (cx->mode == ORC_MODE_REFERENCE) {
            if (ob->nnodes) bvh_ref(ob, 0, r, cx, &h);
            else hit_clear(&h);
        } else {
            hit_clear(&h);
            if (ob->nnodes) {
                int idx[3];
                perm_indices(r->d, idx);
                int behind_ok = fabs(get(r->d, idx[2])) >= 0.01;
                pruned_best pb = {INFINITY, -1, best->valid ? best->distance : INFINITY};
                bvh_pruned(ob, 0, r, cx, behind_ok, &pb);
                if (pb.leaf >= 0) {
                    triangle_intersect(ob->verts + 9 * pb.leaf, ob->norms + 9 * pb.leaf, r, &h);
                    h.primitive = pb.leaf;
                    h.material = ob->material;
                }
            }
        }
        if (!h.valid) continue;
        h.object = oi;
        if (!best->valid || best->distance > h.distance) *best = h;
    }
    if (best->valid) cx->cnt->closest_hits++;
}

int orc_trace(const orc_scene* s, int64_t n, const double* origins, const double* dirs, int32_t mode, orc_hit* out,
              orc_counters* counters) {
    orc_counters local = {0};
    trace_ctx cx = {counters ? counters : &local, mode, 1e-9 * (s->extent + 1.0), 1e-6 * (s->extent + 1.0)};
    for (int64_t i = 0; i < n; ++i) {
        ray r = {ld(origins + 3 * i), ld(dirs + 3 * i)};
        sample_scene(s, &r, &cx, &out[i]);
    }
    return 0;
}

/* ======================================================================================== */
/* Materials (src/materials/) and the integrator                                              */
/* ======================================================================================== */
typedef struct photon {
    double wavelength, intensity;
} photon;

static double mat_colour(const orc_material* m, double wl) {
    return orc_spectrum_intensity(m->shortest, m->longest, m->n, m->s, wl);
}

#define ORC_PI 3.14159265358979323846 /* std::f64::consts::PI */

/* CosineWeightedHemisphere::value (random_distributions/cosine_weighted_hemisphere.rs:20-29)
 * over UnitDisc::value (unit_disc.rs:28-40) over UniformSquare::value (uniform_square.rs:21-26):
 * corner (-1, -1) + (Open01, Open01) * 2, x drawn first */
static v3 cosine_weighted_hemisphere(orc_rng* rng) {
    double ux = rng_open01(rng);
    double uy = rng_open01(rng);
    double ox = -1.0 + ux * 2.0, oy = -1.0 + uy * 2.0;
    double px = ox, py = oy;
    if (!(ox == 0.0 && oy == 0.0)) {
        double radius, angle;
        if (fabs(ox) > fabs(oy)) {
            radius = ox;
            angle = ((ORC_PI / 4.0) * oy) / ox;
        } else {
            radius = oy;
            angle = ORC_PI / 2.0 - ((ORC_PI / 4.0) * ox) / oy;
        }
        px = cos(angle) * radius;
        py = sin(angle) * radius;
    }
    return mk(px, py, sqrt(fmax(0.0, 1.0 - px * px - py * py)));
}
/* CosineWeightedHemisphere::pdf (cosine_weighted_hemisphere.rs:31-33) */
static double cosine_weighted_pdf(v3 v) { return sqrt(v.x * v.x + v.y * v.y) / ORC_PI; }

/* smooth_transparent_dialectric.rs:15-62 */
typedef struct fresnel_result {
    v3 rdir, tdir;
    double R, T;
} fresnel_result;
static fresnel_result fresnel(v3 w_i, double eta1, double eta2) {
    fresnel_result f;
    v3 normal = w_i.z > 0.0 ? mk(0.0, 0.0, 1.0) : mk(-0.0, -0.0, -1.0); /* -Vec3::unit_z() */
    f.rdir = mk(-w_i.x, -w_i.y, w_i.z);
    double r = eta1 / eta2;
    double c1 = dot(normal, w_i);
    double c2sq = 1.0 - r * r * (1.0 - c1 * c1);
    if (c2sq >= 0.0) {
        double c2 = sqrt(c2sq);
        double rpar = (eta1 * c2 - eta2 * c1) / (eta1 * c2 + eta2 * c1);
        double rper = (eta1 * c1 - eta2 * c2) / (eta1 * c1 + eta2 * c2);
        f.R = 0.5 * (rpar * rpar + rper * rper);
        double k = r * c1 - c2;
        f.tdir = normalize(mk(-r * w_i.x + k * normal.x, -r * w_i.y + k * normal.y, -r * w_i.z + k * normal.z));
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
static fresnel_result dielectric_fresnel(const orc_material* m, v3 w_i, double wl) {
    double eta = orc_spectrum_intensity(m->shortest, m->longest, m->n, m->s, wl);
    return w_i.z >= 0.0 ? fresnel(w_i, 1.0, eta) : fresnel(w_i, eta, 1.0);
}

/* lambertian_material.rs:36-59 / reflective_material.rs:42-47 / Material::sample's default for
 * Phong (materials/mod.rs:28-33) / smooth_transparent_dialectric.rs:97-114 */
static void material_sample(const orc_material* m, v3 w_i, double wl, orc_rng* rng, v3* w_o, double* pdf) {
    if (m->kind == ORC_MATERIAL_REFLECTIVE) {
        *w_o = mk(-w_i.x, -w_i.y, w_i.z);
        *pdf = 1.0;
        return;
    }
    if (m->kind == ORC_MATERIAL_PHONG) {
        *w_o = cosine_weighted_hemisphere(rng);
        *pdf = cosine_weighted_pdf(*w_o);
        return;
    }
    if (m->kind == ORC_MATERIAL_DIELECTRIC) {
        fresnel_result f = dielectric_fresnel(m, w_i, wl);
        *pdf = 0.5;
        if (f.T <= 0.0000000001) *w_o = f.rdir;
        else if (f.R <= 0.0000000001 || rng_bool(rng)) *w_o = f.tdir; /* random() only if needed */
        else *w_o = f.rdir;
        return;
    }
    double x = 2.0 * rng_open01(rng) - 1.0;
    double y = 2.0 * rng_open01(rng) - 1.0;
    v3 w = mk(x, y, 0.0);
    while (dot(w, w) > 1.0) {
        x = 2.0 * rng_open01(rng) - 1.0;
        y = 2.0 * rng_open01(rng) - 1.0;
        w = mk(x, y, 0.0);
    }
    w.z = fmax(sqrt(1.0 - w.x * w.x - w.y * w.y), 0.0);
    double cos_theta = dot(w, mk(0.0, 0.0, 1.0));
    double sin_theta = sqrt(1.0 - cos_theta * cos_theta);
    *w_o = normalize(w);
    *pdf = (cos_theta * sin_theta) / 3.14159265358979323846; /* std::f64::consts::PI */
}

/* lambertian_material.rs:27-34 / reflective_material.rs:15-40 */
static photon material_bsdf(const orc_material* m, v3 w_o, v3 w_i, photon in) {
    photon out;
    if (m->kind == ORC_MATERIAL_REFLECTIVE) {
        if (w_i.z <= 0.0 || w_o.z <= 0.0) {
            out.wavelength = in.wavelength;
            out.intensity = 0.0;
            return out;
        }
        v3 refl = mk(-w_o.x, -w_o.y, w_o.z);
        out.wavelength = in.wavelength;
        out.intensity = in.intensity * mat_colour(m, in.wavelength);
        out.intensity *= m->diffuse;
        double sigma = 0.05, two = 2.0;
        double c = dot(w_i, refl);
        c = c < 0.0 ? 0.0 : (c > 1.0 ? 1.0 : c); /* f64::clamp keeps NaN */
        double theta = acos(fabs(c));
        double f = m->reflection * exp(-(pow(theta, two)) / (two * sigma * sigma));
        out.intensity = out.intensity * (1.0 - f) + f;
        return out;
    }
    if (m->kind == ORC_MATERIAL_PHONG) { /* phong_material.rs:17-36 */
        out.wavelength = in.wavelength;
        if (w_i.z < 0.0 || w_o.z < 0.0) {
            out.intensity = 0.0;
            return out;
        }
        v3 refl = mk(-w_i.x, -w_i.y, w_i.z);
        out.intensity = (in.intensity * mat_colour(m, in.wavelength)) * m->diffuse +
                        pow(fabs(dot(w_o, refl)), m->smoothness) * (m->reflection / dot(w_i, mk(0.0, 0.0, 1.0)));
        return out;
    }
    if (m->kind == ORC_MATERIAL_DIELECTRIC) { /* smooth_transparent_dialectric.rs:79-95 */
        fresnel_result f = dielectric_fresnel(m, w_i, in.wavelength);
        v3 dr = sub(w_o, f.rdir), dt = sub(w_o, f.tdir);
        out.wavelength = in.wavelength;
        if (dot(dr, dr) < 0.0000000001) out.intensity = in.intensity * f.R;
        else if (dot(dt, dt) < 0.0000000001) out.intensity = in.intensity * f.T;
        else out.intensity = 0.0;
        return out;
    }
    out.wavelength = in.wavelength;
    out.intensity = in.intensity * mat_colour(m, in.wavelength);
    out.intensity *= m->diffuse;
    return out;
}

typedef struct path_ctx {
    const orc_scene* s;
    trace_ctx* cx;
    orc_rng* rng;
    int bounces;
    int limit_hit;
    int error;
} path_ctx;

/* simple_random_integrator.rs:12-55 */
static photon integrate(path_ctx* pc, const orc_hit* info, photon ph, int limit) {
    photon zero = {0.0, 0.0};
    if (limit == 0) {
        pc->limit_hit = 1;
        return zero;
    }
    m3 world_to_bsdf = from_rows(ld(info->tangent), ld(info->cotangent), ld(info->normal));
    m3 bsdf_to_world;
    if (!try_inverse(&world_to_bsdf, &bsdf_to_world)) { /* the reference panics here */
        pc->error = 1;
        return zero;
    }
    v3 w_i = mul_mv(&world_to_bsdf, ld(info->retro));
    const orc_material* m = &pc->s->mats[info->material];
    v3 w_o;
    double pdf;
    material_sample(m, w_i, ph.wavelength, pc->rng, &w_o, &pdf);
    v3 wo_world = mul_mv(&bsdf_to_world, w_o);
    ray r0 = ray_new(ld(info->location), wo_world);
    ray r = ray_bias(&r0, 0.0000001);
    pc->bounces++;
    orc_hit next;
    sample_scene(pc->s, &r, pc->cx, &next);
    photon below;
    if (!next.valid) {
        below.wavelength = ph.wavelength;
        double w[3];
        st(w, wo_world);
        below.intensity = orc_sky_intensity(w, ph.wavelength);
    } else {
        below = integrate(pc, &next, ph, limit - 1);
    }
    below.intensity = below.intensity * pdf;
    below.intensity = below.intensity * fabs(dot(wo_world, ld(info->normal)));
    return material_bsdf(m, w_o, w_i, below);
}

/* whitted_integrator.rs:20-87.  The continuation ray at recursion limit 0 is not traced: the
 * reference traces it and then discards it (`if recursion_limit > 0 ... else scale 0`), which
 * changes no value; the bounce count records only traced continuations. */
static photon whitted(path_ctx* pc, const orc_hit* info, photon ph, int limit) {
    const orc_scene* s = pc->s;
    photon zero = {ph.wavelength, 0.0};
    m3 w2b = from_rows(ld(info->tangent), ld(info->cotangent), ld(info->normal));
    m3 b2w;
    if (!try_inverse(&w2b, &b2w)) { /* "Expected matrix to be invertable." */
        pc->error = 1;
        return zero;
    }
    const orc_material* m = &s->mats[info->material];
    v3 w_ret = mul_mv(&w2b, ld(info->retro));
    /* material.sample is evaluated when the iterator chain is built, before any light term */
    v3 dir;
    double pdf;
    material_sample(m, w_ret, ph.wavelength, pc->rng, &dir, &pdf);
    double acc = ph.intensity; /* fold(photon.clone(), ...) */
    for (int j = 0; j < s->nlights; ++j) {
        ray r0 = ray_new(ld(info->location), s->light_dir[j]);
        ray r = ray_bias(&r0, 0.0000001);
        orc_hit sh;
        sample_scene(s, &r, pc->cx, &sh);
        double term;
        if (sh.valid) {
            term = orc_spectrum_intensity(s->ambient.shortest, s->ambient.longest, s->ambient.n, s->ambient.s,
                                          ph.wavelength); /* ambient_light.emit_photon */
        } else {
            const orc_material* L = &s->light[j];
            photon in = {ph.wavelength, orc_spectrum_intensity(L->shortest, L->longest, L->n, L->s, ph.wavelength)};
            in.intensity = in.intensity * fabs(dot(s->light_dir[j], ld(info->normal)));
            term = material_bsdf(m, w_ret, mul_mv(&w2b, s->light_dir[j]), in).intensity;
        }
        acc = acc + term;
    }
    if (limit > 0) {
        v3 wd = mul_mv(&b2w, dir);
        ray c0 = ray_new(ld(info->location), wd);
        ray c = ray_bias(&c0, 0.0000001);
        pc->bounces++;
        orc_hit next;
        sample_scene(s, &c, pc->cx, &next);
        if (next.valid) {
            photon below = whitted(pc, &next, ph, limit - 1);
            photon out = material_bsdf(m, w_ret, dir, below);
            acc = acc + out.intensity * fabs(dot(wd, ld(info->normal)));
        } else {
            acc = acc + ph.intensity * 0.0;
        }
    } else {
        pc->limit_hit = 1;
        acc = acc + ph.intensity * 0.0;
    }
    photon out = {ph.wavelength, acc};
    return out;
}

int orc_scene_set_whitted(orc_scene* s, double amb_shortest, double amb_longest, int32_t amb_n,
                          const double* amb_samples, int32_t nlights, const double* dirs, const double* shortest,
                          const double* longest, const int32_t* n, const double* samples) {
    if (nlights < 0 || nlights > 16 || amb_n < 1 || amb_n > 64) return -1;
    s->whitted = 1;
    memset(&s->ambient, 0, sizeof s->ambient);
    s->ambient.shortest = amb_shortest;
    s->ambient.longest = amb_longest;
    s->ambient.n = amb_n;
    memcpy(s->ambient.s, amb_samples, sizeof(double) * amb_n);
    s->nlights = nlights;
    for (int j = 0; j < nlights; ++j) {
        if (n[j] < 1 || n[j] > 64) return -1;
        s->light_dir[j] = ld(dirs + 3 * j);
        memset(&s->light[j], 0, sizeof s->light[j]);
        s->light[j].shortest = shortest[j];
        s->light[j].longest = longest[j];
        s->light[j].n = n[j];
        memcpy(s->light[j].s, samples + 64 * j, sizeof(double) * n[j]);
    }
    return 0;
}

/* One sample of one pixel: the body of camera.rs:105-127 */
static void render_one(const orc_scene* s, trace_ctx* cx, uint64_t height, uint64_t width, uint64_t row, uint64_t col,
                       uint64_t seed, uint64_t sample, orc_sample_record* rec) {
    orc_rng rng = {orc_stream_base(seed, row * width + col, sample), 0};
    double cam[3], o[3], d[3];
    st(cam, s->camera);
    double ux = rng_standard(&rng); /* x's scale() is evaluated first (camera.rs:56-62) */
    double uy = rng_standard(&rng);
    orc_ray_for_pixel(cam, width, height, row, col, ux, uy, o, d);
    ray r = {ld(o), ld(d)};
    orc_hit hit;
    sample_scene(s, &r, cx, &hit);
    photon ph = {0.0, 0.0};
    memset(rec, 0, sizeof *rec);
    if (hit.valid) {
        rec->flags |= 1;
        photon start = {SHORTEST_VISIBLE + (LONGEST_VISIBLE - SHORTEST_VISIBLE) * rng_standard(&rng), 0.0};
        path_ctx pc = {s, cx, &rng, 0, 0, 0};
        ph = s->whitted ? whitted(&pc, &hit, start, 128) : integrate(&pc, &hit, start, 128);
        rec->bounces = pc.bounces;
        if (pc.limit_hit) rec->flags |= 2;
        if (pc.error) { rec->flags |= 4; cx->cnt->errors++; }
    }
    cx->cnt->samples++;
    rec->wavelength = ph.wavelength;
    rec->intensity = ph.intensity;
    double c[3];
    orc_colour_xyz_for_wavelength(ph.wavelength, c);
    double I = ph.intensity * (LONGEST_VISIBLE - SHORTEST_VISIBLE); /* photon.rs:26-28, camera.rs:121-126 */
    for (int k = 0; k < 3; ++k) rec->xyz[k] = c[k] * I;
}

/* ---- threaded drivers ---- */
typedef struct job {
    const orc_scene* s;
    uint64_t c0, c1, r0, r1, h, w;
    uint32_t spp;
    uint64_t seed, first;
    int mode;
    int nthreads, tid;
    double *colour, *sum, *bias, *weight, *wbias;
    orc_sample_record* recs;
    orc_counters cnt;
} job;

static void* tile_worker(void* arg) {
    job* J = (job*)arg;
    trace_ctx cx = {&J->cnt, J->mode, 1e-9 * (J->s->extent + 1.0), 1e-6 * (J->s->extent + 1.0)};
    uint64_t tw = J->c1 - J->c0;
    for (uint64_t rr = J->r0 + (uint64_t)J->tid; rr < J->r1; rr += (uint64_t)J->nthreads) {
        for (uint64_t cc = J->c0; cc < J->c1; ++cc) {
            uint64_t pi = (rr - J->r0) * tw + (cc - J->c0);
            for (uint32_t k = 0; k < J->spp; ++k) {
                orc_sample_record rec;
                render_one(J->s, &cx, J->h, J->w, rr, cc, J->seed, J->first + k, &rec);
                if (J->recs) {
                    J->recs[pi * J->spp + k] = rec;
                } else {
                    /* update_pixel(row, column, photon x 360, 1.0): the x360 is folded into the intensity */
                    orc_update_pixel(J->colour + 3 * pi, J->sum + 3 * pi, J->bias + 3 * pi, J->weight + pi,
                                     J->wbias + pi, rec.wavelength, rec.intensity * 360.0, 1.0);
                }
            }
        }
    }
    return NULL;
}

static int run_jobs(job* proto, int nthreads, orc_counters* counters) {
    if (nthreads < 1) nthreads = 1;
    job* jobs = (job*)calloc((size_t)nthreads, sizeof(job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = *proto;
        jobs[t].nthreads = nthreads;
        jobs[t].tid = t;
        memset(&jobs[t].cnt, 0, sizeof(orc_counters));
        if (nthreads == 1) tile_worker(&jobs[t]);
        else pthread_create(&th[t], NULL, tile_worker, &jobs[t]);
    }
    orc_counters tot = {0};
    for (int t = 0; t < nthreads; ++t) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        tot.box_tests += jobs[t].cnt.box_tests;
        tot.triangle_tests += jobs[t].cnt.triangle_tests;
        tot.rays += jobs[t].cnt.rays;
        tot.samples += jobs[t].cnt.samples;
        tot.closest_hits += jobs[t].cnt.closest_hits;
        tot.errors += jobs[t].cnt.errors;
    }
    if (counters) *counters = tot;
    free(jobs);
    free(th);
    return tot.errors ? 1 : 0;
}

int orc_render_tile(const orc_scene* s, uint64_t c0, uint64_t c1, uint64_t r0, uint64_t r1, uint64_t h, uint64_t w,
                    uint32_t spp, uint64_t seed, uint64_t first, int32_t mode, int32_t nthreads, int32_t accumulate,
                    double* colour, double* sum, double* bias, double* weight, double* wbias, orc_counters* counters) {
    if (c1 < c0 || r1 < r0 || c1 > w || r1 > h) return -1;
    uint64_t n = (c1 - c0) * (r1 - r0);
    if (!accumulate) {
        memset(colour, 0, sizeof(double) * 3 * n);
        memset(sum, 0, sizeof(double) * 3 * n);
        memset(bias, 0, sizeof(double) * 3 * n);
        memset(weight, 0, sizeof(double) * n);
        memset(wbias, 0, sizeof(double) * n);
    }
    job J;
    memset(&J, 0, sizeof J);
    J.s = s; J.c0 = c0; J.c1 = c1; J.r0 = r0; J.r1 = r1; J.h = h; J.w = w; J.spp = spp; J.seed = seed;
    J.first = first; J.mode = mode; J.colour = colour; J.sum = sum; J.bias = bias; J.weight = weight; J.wbias = wbias;
    return run_jobs(&J, nthreads, counters);
}

int orc_render_samples(const orc_scene* s, uint64_t c0, uint64_t c1, uint64_t r0, uint64_t r1, uint64_t h, uint64_t w,
                       uint32_t spp, uint64_t seed, uint64_t first, int32_t mode, int32_t nthreads,
                       orc_sample_record* out) {
    if (c1 < c0 || r1 < r0 || c1 > w || r1 > h) return -1;
    job J;
    memset(&J, 0, sizeof J);
    J.s = s; J.c0 = c0; J.c1 = c1; J.r0 = r0; J.r1 = r1; J.h = h; J.w = w; J.spp = spp; J.seed = seed;
    J.first = first; J.mode = mode; J.recs = out;
    return run_jobs(&J, nthreads, NULL);
}

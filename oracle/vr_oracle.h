/*
 * vr_oracle.h -- CPU restatement of vanrijn's per-pixel hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This library is the parity checker for the MI355X path.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product (vanrijn_amd/) never links, includes
 * or calls anything under oracle/.
 *
 * Parity status (see DESIGN.md section "Oracle"):
 *   - PINNED by the reference's own known-answer tests, ported in tests/test_oracle_kats.py:
 *     triangle intersection (src/raycasting/triangle.rs:396-496 + properties :531-915),
 *     AABB slab test (src/raycasting/axis_aligned_bounding_box.rs:85-123), sphere
 *     (src/raycasting/sphere.rs:112-184), plane (src/raycasting/plane.rs:118-297),
 *     spectrum lookup (src/colour/spectrum.rs:427-488), CIE round trip
 *     (src/colour/colour_xyz.rs:127-133), accumulation buffer (src/accumulation_buffer.rs:127-327),
 *     Mat3 (src/math/mat3.rs:185-357), camera (src/camera.rs:143-182), Ray
 *     (src/raycasting/mod.rs:155-181), change of basis (src/util/algebra_utils.rs:16-49),
 *     Interval (src/util/interval.rs:97-327), util BoundingBox
 *     (src/util/axis_aligned_bounding_box.rs:108-239).
 *   - UNPINNED (the reference has no tests for them and cannot be built here: no Rust
 *     toolchain): BVH traversal, sampler, integrator, materials,
 *     reflection_from_linear_rgb, CMF values, whole images.  Restated line by line instead.
 *   - The reference draws from rand 0.7's ThreadRng (ChaCha, reseeded from OS entropy, cannot be
 *     seeded: SURVEY.md F4).  The oracle and the product both draw from the counter-based
 *     "vr-hash32 v2" stream defined below; the u64 -> f64 maps follow rand 0.7's Standard and
 *     Open01 (parity of those maps: unpinned, no reference test covers them).
 *
 * Build: oracle/Makefile (gcc, -O2 -ffp-contract=off: Rust never contracts a*b+c into an FMA).
 */
#ifndef VR_ORACLE_H
#define VR_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- random stream (shared definition with the product, restated independently there) ---- */
uint64_t orc_mix64(uint64_t z);
uint32_t orc_hash32(uint32_t x);
uint64_t orc_stream_base(uint64_t seed, uint64_t pixel_index, uint64_t sample_index);
uint64_t orc_stream_draw(uint64_t base, uint64_t k);
double orc_u64_to_standard(uint64_t u); /* rand 0.7 Standard f64: [0,1) */
double orc_u64_to_open01(uint64_t u);   /* rand 0.7 Open01 f64: (0,1) */

/* ---- low-level pieces, exported for the reference's known-answer tests ---- */
typedef struct orc_hit {
    int32_t valid;
    int32_t object;     /* index into the scene object list */
    int64_t primitive;  /* primitive-list position, or BVH leaf (in-order) position */
    int32_t material;
    int32_t pad;
    double distance;
    double location[3];
    double normal[3];
    double tangent[3];
    double cotangent[3];
    double retro[3];
} orc_hit;

void orc_normalize(const double v[3], double out[3]);
int orc_bbox_intersect(const double bmin[3], const double bmax[3], const double o[3], const double d[3]);
void orc_triangle_intersect(const double v[9], const double n[9], const double o[3], const double d[3], orc_hit* out);
void orc_sphere_intersect(const double centre[3], double radius, const double o[3], const double d[3], orc_hit* out);
void orc_plane_new(const double normal_in[3], double out_n[3], double out_t[3], double out_c[3]);
void orc_plane_intersect(const double n[3], const double t[3], const double c[3], double dist, const double o[3],
                         const double d[3], orc_hit* out);
int orc_mat3_inverse(const double m[9], double out[9]); /* cofactor^T * det, as mat3.rs:111-118 */
double orc_mat3_determinant(const double m[9]);
double orc_mat3_first_minor(const double m[9], int32_t row, int32_t column);
void orc_mat3_cofactor_matrix(const double m[9], double out[9]);
void orc_mat3_transpose(const double m[9], double out[9]);
void orc_mat3_mul(const double a[9], const double b[9], double out[9]);
void orc_mat3_mul_vec(const double m[9], const double v[3], double out[3]);
void orc_change_of_basis(const double x[3], const double y[3], const double z[3], double out[9]);
/* Interval as {min, max}; util BoundingBox as {min x, max x, min y, max y, min z, max z} */
void orc_interval_new(double a, double b, double out[2]);
void orc_interval_union(const double a[2], const double b[2], double out[2]);
void orc_interval_intersection(const double a[2], const double b[2], double out[2]);
void orc_interval_expand(const double a[2], double v, double out[2]);
int orc_interval_is_empty(const double a[2]);
int orc_interval_is_degenerate(const double a[2]);
int orc_interval_contains(const double a[2], double v);
void orc_bbox_from_corners(const double a[3], const double b[3], double out[6]);
void orc_bbox_from_points(int64_t n, const double* pts, double out[6]);
void orc_bbox_union(const double a[6], const double b[6], double out[6]);
int orc_bbox_contains_point(const double b[6], const double p[3]);
int orc_bbox_largest_dimension(const double b[6]);
void orc_ray_new(const double o[3], const double d[3], double out_o[3], double out_d[3]);
void orc_ray_point_at(const double o[3], const double d[3], double t, double out[3]);
double orc_spectrum_intensity(double shortest, double longest, int32_t n, const double* samples, double wavelength);
void orc_reflection_from_linear_rgb(double r, double g, double b, double out[32]);
void orc_colour_xyz_for_wavelength(double wavelength, double out[3]);
void orc_colour_xyz_to_linear_rgb(const double xyz[3], double rgb[3]);
void orc_colour_xyz_from_linear_rgb(const double rgb[3], double xyz[3]);
double orc_sky_intensity(const double w[3], double wavelength);
/* ImageSampler::ray_for_pixel with the two jitter draws given explicitly */
void orc_ray_for_pixel(const double cam[3], uint64_t width, uint64_t height, uint64_t row, uint64_t column, double u_x,
                       double u_y, double o[3], double d[3]);
/* AccumulationBuffer::update_pixel on one pixel's state */
void orc_update_pixel(double colour[3], double sum[3], double bias[3], double* weight, double* weight_bias,
                      double wavelength, double intensity, double w);
/* AccumulationBuffer::merge_tile; dst is [dst_h][dst_w], src is [tile rows][tile cols] */
void orc_merge_tile(uint64_t dst_width, double* dst_colour, double* dst_weight, uint64_t start_row,
                    uint64_t start_column, uint64_t tile_h, uint64_t tile_w, const double* src_colour,
                    const double* src_weight);

/* ---- scene ---- */
typedef struct orc_scene orc_scene;
enum { ORC_MATERIAL_LAMBERTIAN = 0, ORC_MATERIAL_REFLECTIVE = 1, ORC_MATERIAL_PHONG = 2, ORC_MATERIAL_DIELECTRIC = 3 };
enum { ORC_PRIM_PLANE = 0, ORC_PRIM_SPHERE = 1 };

orc_scene* orc_scene_new(const double camera[3]);
void orc_scene_free(orc_scene*);
int orc_scene_add_material(orc_scene*, int32_t kind, double shortest, double longest, int32_t n, const double* samples,
                           double diffuse, double reflection, double smoothness);
/* One object = Vec<Box<dyn Primitive>> (vec_aggregate.rs:11-22): kinds/materials/vecs(3 each)/scalars */
int orc_scene_add_primitive_list(orc_scene*, int32_t count, const int32_t* kinds, const int32_t* materials,
                                 const double* vecs, const double* scalars);
/* One object = BoundingVolumeHierarchy::build over a triangle mesh (bounding_volume_hierarchy.rs:49-74) */
int orc_scene_add_mesh(orc_scene*, int64_t triangle_count, const double* vertices, const double* normals,
                       int32_t material);
/* leaf (in-order) order of a mesh BVH: out[i] = original triangle index of leaf i */
int orc_scene_mesh_leaf_order(const orc_scene*, int32_t object, int64_t* out);
int orc_scene_mesh_depth(const orc_scene*, int32_t object);

enum { ORC_MODE_REFERENCE = 0, ORC_MODE_PRUNED = 1 };

typedef struct orc_counters {
    uint64_t box_tests;
    uint64_t triangle_tests;
    uint64_t rays;
    uint64_t samples;
    uint64_t closest_hits; /* hits whose shading data (normals) is read */
    uint64_t errors;       /* singular basis (the reference panics) */
} orc_counters;

/* Sampler::sample for a batch of rays (directions used as given). */
int orc_trace(const orc_scene*, int64_t n, const double* origins, const double* directions, int32_t mode,
              orc_hit* out, orc_counters* counters);

/* Per-(pixel, sample) record for decision-identity checks. */
typedef struct orc_sample_record {
    double wavelength; /* final photon wavelength (0 on miss or recursion limit) */
    double intensity;  /* final photon intensity, before the 1/pdf (x360) scale */
    double xyz[3];     /* ColourXyz::from_photon(photon.scale_intensity(360)) */
    int32_t bounces;   /* bounce rays traced (0..128) */
    int32_t flags;     /* bit0 camera hit, bit1 recursion limit, bit2 singular basis */
} orc_sample_record;

/* partial_render_scene generalised: spp samples per pixel of the tile, each sample exactly as
 * one call of partial_render_scene (camera.rs:95-130), accumulated with update_pixel into the
 * tile buffers ([tile_h][tile_w][3] / [tile_h][tile_w]).  accumulate=0 clears them first. */
int orc_render_tile(const orc_scene*, uint64_t start_column, uint64_t end_column, uint64_t start_row,
                    uint64_t end_row, uint64_t height, uint64_t width, uint32_t spp, uint64_t seed,
                    uint64_t first_sample, int32_t mode, int32_t nthreads, int32_t accumulate, double* colour,
                    double* colour_sum, double* colour_bias, double* weight, double* weight_bias,
                    orc_counters* counters);
int orc_render_samples(const orc_scene*, uint64_t start_column, uint64_t end_column, uint64_t start_row,
                       uint64_t end_row, uint64_t height, uint64_t width, uint32_t spp, uint64_t seed,
                       uint64_t first_sample, int32_t mode, int32_t nthreads, orc_sample_record* out);

/* Render with WhittedIntegrator (whitted_integrator.rs:15-87) instead of SimpleRandomIntegrator:
 * ambient spectrum + nlights (<= 16) directional lights (dirs [n][3]; spectra: samples [n][64]). */
int orc_scene_set_whitted(orc_scene*, double amb_shortest, double amb_longest, int32_t amb_n,
                          const double* amb_samples, int32_t nlights, const double* dirs, const double* shortest,
                          const double* longest, const int32_t* n, const double* samples);

/* AccumulationBuffer::to_image_rgb_u8(&ClampingToneMapper) on the colour buffer [n][3]. */
void orc_tone_map(const double* colour, uint64_t n, uint8_t* rgb);

#ifdef __cplusplus
}
#endif
#endif

/*
 * vanrijn_amd.h -- C ABI of the MI355X (gfx950) path-tracing core.
 *
 * Drop-in boundary for vanrijn's per-pixel hot path.  The reference's boundary is
 *     pub fn partial_render_scene(scene: &Scene, tile: Tile, height: usize, width: usize)
 *         -> AccumulationBuffer                                   (src/camera.rs:95-130)
 * called concurrently from rayon workers in src/main.rs:204 and from benches/simple_scene.rs:45.
 * Every entry point below names the reference interface it replaces.  Plain pointers and sizes
 * only; no HIP or torch types in the signatures (streams are passed as void*).  A Rust binding
 * (extern "C" block) is shown in INTEGRATION.md.
 *
 * Conventions
 *   - All floating point is IEEE binary64, as in the reference (everything on the path is f64).
 *   - Return value: VR_OK (0) or a negative vr_status.  The message of the last failure on the
 *     calling thread is in vr_last_error().  Nothing unwinds across the ABI; where the reference
 *     panics (singular shading basis, out-of-range tile) the call returns an error instead.
 *   - A vr_scene is immutable after creation and may be shared by any number of threads;
 *     render calls are re-entrant.  Each call holds its own stream, staging buffer, work-queue
 *     counter and device error word for its duration (a per-scene pool of call contexts), so
 *     concurrent calls neither serialise on shared scratch nor see each other's errors
 *     (tests/test_gpu_concurrency.py).
 *   - Errors found on the device (the singular shading basis where the reference panics,
 *     simple_random_integrator.rs:26-31) belong to the call that found them: synchronous entry
 *     points return them; the asynchronous vr_render_tile_device records them in a sticky word of
 *     its stream, returned by the next vr_stream_check_error (or timed launch) on that stream.
 */
#ifndef VANRIJN_AMD_H
#define VANRIJN_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VR_ABI_VERSION 10
#define VR_MAX_SPECTRUM_SAMPLES 64
#define VR_RECURSION_LIMIT 128 /* camera.rs:69 */

typedef enum vr_status {
    VR_OK = 0,
    VR_ERROR_INVALID_ARGUMENT = -1,
    VR_ERROR_OUT_OF_MEMORY = -2,
    VR_ERROR_DEVICE = -3,          /* a HIP call failed */
    VR_ERROR_NO_DEVICE = -4,       /* no gfx950 device visible */
    VR_ERROR_SINGULAR_BASIS = -5,  /* simple_random_integrator.rs:26-31 would panic ("expect") */
    VR_ERROR_IO = -6,              /* load_obj: std::io::Error (src/mesh.rs:74-77) */
    VR_ERROR_UNSUPPORTED = -7,     /* e.g. BVH deeper than the traversal stack */
    VR_ERROR_HOST_ONLY = -8        /* render call on a scene created with VR_SCENE_HOST_ONLY */
} vr_status;

typedef struct vr_vec3 {
    double x, y, z;
} vr_vec3; /* math::Vec3 (src/math/vec3.rs:8-10) */

/* colour::Spectrum (src/colour/spectrum.rs:5-10): samples linearly interpolated over
 * [shortest_wavelength, longest_wavelength], zero outside. */
typedef struct vr_spectrum {
    double shortest_wavelength;
    double longest_wavelength;
    uint32_t sample_count; /* 2 .. VR_MAX_SPECTRUM_SAMPLES */
    const double* samples;
} vr_spectrum;

typedef enum vr_material_kind {
    VR_MATERIAL_LAMBERTIAN = 0, /* materials/lambertian_material.rs:12-60 */
    VR_MATERIAL_REFLECTIVE = 1, /* materials/reflective_material.rs:8-48 */
    VR_MATERIAL_PHONG = 2,      /* materials/phong_material.rs:8-37 (sample: materials/mod.rs:28-33) */
    VR_MATERIAL_DIELECTRIC = 3  /* materials/smooth_transparent_dialectric.rs:64-115 (colour = eta) */
} vr_material_kind;

typedef struct vr_material_desc {
    int32_t kind;
    uint32_t reserved;
    vr_spectrum colour;         /* the refractive index eta(lambda) for the dielectric */
    double diffuse_strength;    /* Lambertian, reflective, Phong */
    double reflection_strength; /* reflective; Phong's specular_strength */
    double smoothness;          /* Phong only */
} vr_material_desc;

typedef enum vr_primitive_kind {
    VR_PRIMITIVE_PLANE = 0, /* raycasting/plane.rs:18-31: vector = normal (normalised here, as Plane::new), scalar = distance_from_origin */
    VR_PRIMITIVE_SPHERE = 1 /* raycasting/sphere.rs:15-23: vector = centre, scalar = radius */
} vr_primitive_kind;

typedef struct vr_primitive_desc {
    int32_t kind;
    uint32_t material;
    vr_vec3 vector;
    double scalar;
} vr_primitive_desc;

/* A triangle mesh (Vec<Arc<dyn Primitive>> of raycasting::Triangle, src/raycasting/triangle.rs:8-13).
 * vertices/normals: [triangle][corner 0..2][xyz] doubles; copied by vr_scene_create. */
typedef struct vr_mesh_desc {
    uint64_t triangle_count;
    const double* vertices;
    const double* normals;
    uint32_t material;
    uint32_t reserved;
} vr_mesh_desc;

typedef enum vr_object_kind {
    VR_OBJECT_PRIMITIVE_LIST = 0, /* Box<Vec<Box<dyn Primitive>>> (raycasting/vec_aggregate.rs:11-24) */
    VR_OBJECT_BVH = 1             /* Box<BoundingVolumeHierarchy> (raycasting/bounding_volume_hierarchy.rs:49-74) */
} vr_object_kind;

typedef struct vr_object_desc {
    int32_t kind;
    uint32_t first; /* primitive list: first primitive index; BVH: mesh index */
    uint32_t count; /* primitive list: number of primitives; BVH: must be 1 */
    uint32_t reserved;
} vr_object_desc;

/* scene::Scene (src/scene.rs:5-8): camera_location + objects in order (order decides ties,
 * sampler.rs:9-20). */
/* Integrators.  The reference's partial_render_scene always uses SimpleRandomIntegrator
 * (camera.rs:103); WhittedIntegrator (integrators/whitted_integrator.rs:15-87: directional lights
 * with shadow rays, an ambient term, one sampled continuation per hit) is selectable per scene. */
typedef enum vr_integrator_kind {
    VR_INTEGRATOR_SIMPLE_RANDOM = 0,
    VR_INTEGRATOR_WHITTED = 1
} vr_integrator_kind;

typedef struct vr_directional_light { /* whitted_integrator.rs:10-13 */
    vr_vec3 direction;
    vr_spectrum spectrum;
} vr_directional_light;

typedef struct vr_integrator_desc {
    int32_t kind;
    uint32_t light_count;        /* at most VR_MAX_LIGHTS */
    vr_spectrum ambient_light;   /* Whitted */
    const vr_directional_light* lights;
} vr_integrator_desc;
#define VR_MAX_LIGHTS 16

typedef struct vr_scene_desc {
    vr_vec3 camera_location;
    uint32_t material_count;
    uint32_t primitive_count;
    uint32_t mesh_count;
    uint32_t object_count;
    const vr_material_desc* materials;
    const vr_primitive_desc* primitives;
    const vr_mesh_desc* meshes;
    const vr_object_desc* objects;
    const vr_integrator_desc* integrator; /* NULL: SimpleRandomIntegrator */
} vr_scene_desc;

typedef struct vr_scene vr_scene;

#define VR_SCENE_HOST_ONLY 1u /* build + flatten only, no device upload (inspection, CPU tests) */
/* Build the meshes' BVHs on the device (level-synchronous sorts; the same nodes and leaf order as
 * the host build, bounding_volume_hierarchy.rs:38-74).  Meshes with NaN coordinates use the host
 * build.  Ignored with VR_SCENE_HOST_ONLY. */
#define VR_SCENE_DEVICE_BVH 2u
/* Traverse the reference's own median-split tree instead of the default SAH tree.  Results are
 * identical either way (the closest hit does not depend on the tree; ties follow the reference
 * tree's in-order leaf rank); the device build always produces the reference tree. */
#define VR_SCENE_REFERENCE_BVH 4u
/* Build the default traversal tree on the device as well (ABI 5): the reference's median-split
 * build above gives every triangle its in-order rank (the tie-break), then a binned-SAH binary
 * tree (the host build's algorithm, one workgroup per node and level) is built over the ranked
 * triangles and collapsed to the 4-wide render tree.  Renders are bit-identical to the host-built
 * scene's; only the build time differs.  Implies VR_SCENE_DEVICE_BVH; ignored with
 * VR_SCENE_REFERENCE_BVH or VR_SCENE_HOST_ONLY. */
#define VR_SCENE_DEVICE_SAH 8u
/* Collapse the binary traversal tree to the 4-wide render tree greedily (the largest-area interior
 * child expanded first) instead of by the SAH-optimal dynamic programme.
 * Renders are identical either way; for inspection and the collapse's own tests (ABI 7). */
#define VR_SCENE_GREEDY_COLLAPSE 16u
/* Render with the 64-bit-offset kernels whatever the scene's size (ABI 8).  They are chosen
 * automatically for scenes past the 32-bit load offsets of the default kernels -- 4 GB of triangle
 * records (53.7 M triangles) or 2^25 nodes of the 4-wide tree (vr_scene_needs_wide_offsets); this
 * flag exercises them on small scenes (tests).  Renders are identical either way. */
#define VR_SCENE_WIDE_OFFSETS 32u

/* Replaces building `Scene { camera_location, objects }` + BoundingVolumeHierarchy::build.
 * Copies every input; builds one BVH per mesh with the reference's median split
 * (bounding_volume_hierarchy.rs:38-74; ties in the sort broken by input triangle index);
 * flattens it and uploads it to `device` (HIP ordinal). */
int vr_scene_create(const vr_scene_desc* desc, int32_t device, uint32_t flags, vr_scene** out);
void vr_scene_destroy(vr_scene* scene);

typedef struct vr_scene_info {
    uint64_t triangle_count;
    uint64_t node_count;     /* flattened interior nodes over all BVHs */
    uint32_t max_bvh_depth;  /* levels, root = 1 */
    uint32_t object_count;
    double extent;           /* max |coordinate| of camera and geometry */
    uint64_t device_bytes;   /* scene bytes resident in HBM */
    uint64_t wide_node_count;  /* nodes of the render kernel's 4-wide traversal tree (ABI 3) */
    uint32_t traversal_stack;  /* deepest stack of the 4-wide walk, entries (ABI 3) */
    uint32_t flags;            /* VR_SCENE_INFO_* (ABI 5) */
} vr_scene_info;
/* Every continuation of every path is provably finite (each traced mesh triangle's vertex normals
 * lie strictly on one side of its plane, so the shading basis of triangle.rs:73-78 is finite at any
 * barycentric point; no Phong or dielectric material).  Only then does a path whose throughput is
 * exactly 0 end early; otherwise it is traced to the end, so a later NaN (e.g. the zero normals
 * mesh.rs:37 gives an OBJ without normals) reaches the pixel as the reference's 0 * NaN does
 * (simple_random_integrator.rs:39-53). */
#define VR_SCENE_INFO_NAN_FREE 1u
int vr_scene_get_info(const vr_scene* scene, vr_scene_info* out);
/* BVH leaf (in-order) sequence of mesh `mesh`: out[i] = input triangle index of leaf i. */
int vr_scene_bvh_leaf_order(const vr_scene* scene, uint32_t mesh, uint64_t* out);
/* The scene's flattened BVH interior nodes (all meshes, pre-order per mesh, scene-wide links):
 * node_count records of 128 B = { double box[2][6] (child c: min x, max x, min y, max y, min z,
 * max z); int32 child[2] (>= 0 interior node, < 0 leaf holding triangle ~child); 24 B pad }.
 * For inspection and build-parity tests. */
int vr_scene_bvh_nodes(const vr_scene* scene, void* out_nodes);

/* util::Tile (src/util/tile_iterator.rs:1-7): half-open row/column ranges of the full image. */
typedef struct vr_tile {
    uint64_t start_column, end_column, start_row, end_row;
} vr_tile;

/* AccumulationBuffer (src/accumulation_buffer.rs:6-12), row-major over the tile:
 * colour/colour_sum/colour_bias: [height][width][3] XYZ; weight/weight_bias: [height][width].
 * colour is the running mean (sum * (1/weight)); the *_bias arrays are the Kahan compensation. */
typedef struct vr_accumulation_buffer {
    uint64_t width, height;
    double* colour;
    double* colour_sum;
    double* colour_bias;
    double* weight;
    double* weight_bias;
} vr_accumulation_buffer;

/* Sampling parameters.  Each (pixel, sample) draws its random numbers from the counter-based
 * stream (seed, row*width+column, first_sample + s) ("vr-hash32 v2"), so results do
 * not depend on tiling, launch split or device count.  The stream's index space is 2^32 pixels x 2^32
 * samples: width*height > 2^32 or first_sample + spp > 2^32 returns VR_ERROR_UNSUPPORTED.  Each 64-bit
 * draw is two 32-bit hashes of one 32-bit counter word, so it carries 32 bits of state (a Standard
 * f64 takes one of at most 2^32 values). */
typedef struct vr_render_params {
    vr_tile tile;
    uint64_t height, width; /* full image, as partial_render_scene's height/width */
    uint32_t spp;           /* samples per pixel in this call (partial_render_scene == 1) */
    uint32_t accumulate;    /* 0: start from AccumulationBuffer::new(); 1: continue update_pixel */
    uint64_t seed;
    uint64_t first_sample;
} vr_render_params;

/* Replaces partial_render_scene (camera.rs:95-130) one-for-one: one sample per pixel into a
 * fresh tile buffer (`out` arrays are caller-allocated host memory, tile-sized).  The sample
 * index comes from a per-scene atomic pass counter starting at 0 (seed 0x5EED0001), so concurrent
 * callers get distinct random streams like the reference's thread_rng.  Thread-safe. */
int vr_partial_render_scene(const vr_scene* scene, vr_tile tile, uint64_t height, uint64_t width,
                            vr_accumulation_buffer* out);

/* Generalised form: spp samples per pixel, explicit seed / sample range, host buffers; `buf`
 * is read first when params->accumulate is 1 (update_pixel continuation). */
int vr_render_tile(const vr_scene* scene, const vr_render_params* params, vr_accumulation_buffer* buf);

/* Device-resident form for the multi-GPU path: `state` is a device pointer to the tile's records
 * (ABI 7) -- 8 doubles per pixel in two halves, for the n = tile_width*tile_height pixels in
 * row-major order:
 *     state[4p .. 4p+3]           = {sum X, sum Y, sum Z, weight}        (colour_sum, weight)
 *     state[4n + 4p .. 4n + 4p+3] = {bias X, bias Y, bias Z, weight_bias} (Kahan compensations)
 * The first half is the merge-exact part: records of disjoint sample sets (one per GPU) merge by
 * adding it, in place, with one collective over 32 B per pixel.  `stream` is a hipStream_t (NULL =
 * the null stream) and the call only enqueues work (no host synchronisation). */
typedef struct vr_launch_stats {
    float kernel_ms;          /* HIP-event time of the render kernel launch(es), valid when timed != 0 */
    uint32_t timed;
    uint64_t box_tests;       /* filled only when counters were requested */
    uint64_t node_visits;
    uint64_t triangle_tests;
    uint64_t rays;
    uint64_t shaded_triangle_hits;
    uint64_t samples;
    uint64_t traversal_slots;  /* 64 x wave-level traversal-loop iterations (lane utilisation) */
    uint64_t path_loop_slots;  /* 64 x wave-level path-loop iterations */
    uint64_t exact_box_tests;  /* f32 box tests too close to call, re-run exactly in f64 */
    float reduce_ms;           /* HIP-event time of the ordered per-pixel Kahan reduce(s) (timed) */
    uint32_t passes;           /* render + reduce launches (the staging buffer bounds a launch) */
    uint32_t variant;          /* VR_VARIANT_* bits of the render kernel that ran (ABI 8) */
    uint32_t reserved;
} vr_launch_stats;
#define VR_VARIANT_COOP 1u         /* the cooperative-tail instantiation (small launches, mirror scenes) */
#define VR_VARIANT_WIDE_OFFSETS 2u /* the 64-bit-offset kernels (VR_SCENE_WIDE_OFFSETS) */
#define VR_VARIANT_STACK16 4u      /* 16-bit traversal-stack entries (trees below 65,536 wide nodes; ABI 10) */

#define VR_LAUNCH_TIMED 1u    /* bracket the kernel with HIP events and synchronise at the end */
#define VR_LAUNCH_COUNTERS 2u /* counting build of the kernel (slower), fills the counters */
/* with VR_LAUNCH_TIMED: record the HIP events but return without waiting (stats: passes only); the
 * times are read later by vr_collect_launch_times, so back-to-back timed frames leave the GPU no
 * idle gap for a host round trip (ABI 6).  The caller must collect: a stream holds at most 4096
 * uncollected deferred launches, beyond which the call fails with VR_ERROR_INVALID_ARGUMENT. */
#define VR_LAUNCH_DEFER_TIMES 4u
/* skip the camera-frustum culling of 8x8 pixel blocks (every sample traced): the records are the
 * same bit for bit (tests/test_gpu_cull.py); for tests and A/B measurements (ABI 7) */
#define VR_LAUNCH_NO_CULL 8u
/* no BVH distance culling: every box the ray's line crosses is walked (the reference's exhaustive
 * traversal, bounding_volume_hierarchy.rs:94-120), with the same records bit for bit -- the check
 * that the tie rule does not lean on the culling order (tests/test_gpu_launch_variants.py; ABI 8) */
#define VR_LAUNCH_NO_DIST_CULL 16u
/* no cooperative tail (small launches of scenes with a reflective material otherwise spread a
 * wave's last one or two paths over its lanes): the same records bit for bit (ABI 8) */
#define VR_LAUNCH_NO_COOP 32u
/* cooperative tail without its whole-walk form (the one or two live paths' walks run in coop_step's
 * per-step form only): the same records bit for bit; for tests and A/B measurements (ABI 9) */
#define VR_LAUNCH_NO_LONE_WALK 64u
/* keep 32-bit traversal-stack entries where the tree would allow 16-bit ones: the same records bit for
 * bit; for tests and A/B measurements (ABI 10) */
#define VR_LAUNCH_STACK32 128u

int vr_render_tile_device(const vr_scene* scene, const vr_render_params* params, double* state, void* stream,
                          uint32_t launch_flags, vr_launch_stats* stats);
/* Waits for `stream` and returns the first device error (VR_ERROR_SINGULAR_BASIS) of any
 * vr_render_tile_device launch of `scene` on that stream since the last check, then clears it
 * (ABI 4).  A VR_LAUNCH_TIMED launch performs this check itself. */
int vr_stream_check_error(const vr_scene* scene, void* stream);
/* Waits for the VR_LAUNCH_DEFER_TIMES launches of `scene` on `stream` since the last collection
 * and returns their summed HIP-event times, then forgets them; reports their device errors like
 * vr_stream_check_error (ABI 6). */
typedef struct vr_launch_times {
    double kernel_ms;    /* render kernel, summed over the launches' passes */
    double reduce_ms;    /* ordered per-pixel Kahan reduce, summed */
    uint32_t launches;   /* vr_render_tile_device calls collected */
    uint32_t passes;     /* render + reduce launches in them */
    uint32_t max_passes; /* the most passes of one call */
    uint32_t reserved;
} vr_launch_times;
int vr_collect_launch_times(const vr_scene* scene, void* stream, vr_launch_times* out);
/* Mean XYZ of host-side state records (the layout of vr_render_tile_device; only the sums half is
 * read): colour = colour_sum * (1 / weight) (accumulation_buffer.rs:59).  States of disjoint sample
 * sets (e.g. one per GPU) merge by element-wise addition of the sums half (the cross-GPU reduce),
 * which is what AccumulationBuffer::merge_tile's weighted blend (accumulation_buffer.rs:62-85)
 * computes. */
int vr_resolve_state(const double* state_host, uint64_t pixel_count, double* colour_out);
/* AccumulationBuffer::merge_tile (accumulation_buffer.rs:62-85, the host side of main.rs:214-216):
 * for every pixel of `tile` (full-image coordinates in `dst`), dst colour = blend(dst colour, dst
 * weight, src colour, src weight) = (c1 * w1 + c2 * w2) * (1 / (w1 + w2)); dst weight += src
 * weight.  dst's colour_sum / bias buffers are not touched (as in the reference).  Host only (ABI 4). */
int vr_merge_tile(vr_accumulation_buffer* dst, vr_tile tile, const vr_accumulation_buffer* src);

/* Per-(pixel, sample) records, for decision-identity checks against the oracle. */
typedef struct vr_sample_record {
    double wavelength; /* final photon wavelength (0 on camera miss / recursion limit) */
    double intensity;  /* final photon intensity before the x360 pdf scale */
    double xyz[3];     /* ColourXyz::from_photon of the scaled photon */
    int32_t bounces;   /* bounce rays traced */
    int32_t flags;     /* bit0 camera ray hit, bit1 recursion limit reached, bit2 singular basis */
} vr_sample_record;
int vr_render_samples(const vr_scene* scene, const vr_render_params* params, vr_sample_record* out);

/* Sampler::sample (src/sampler.rs:9-20) for a batch of rays (origins/directions: [n][3], the
 * directions are used as given, as Ray's fields).  Host arrays. */
typedef struct vr_hit_record {
    int32_t valid;
    int32_t object;
    int64_t primitive; /* primitive-list position, or BVH leaf position */
    double distance;
    double location[3];
    double normal[3];
    double tangent[3];
    double cotangent[3];
    double retro[3];
} vr_hit_record;
int vr_trace_rays(const vr_scene* scene, uint64_t n, const double* origins, const double* directions,
                  vr_hit_record* out);

/* Host helpers (scene setup; no device work). */
/* Spectrum::reflection_from_linear_rgb (spectrum.rs:81-165): 32 samples over [380, 720] nm. */
int vr_spectrum_reflection_from_linear_rgb(double red, double green, double blue, double out[32]);
/* Spectrum::intensity_at_wavelength (spectrum.rs:64-79). */
double vr_spectrum_intensity_at_wavelength(const vr_spectrum* spectrum, double wavelength);
/* ColourXyz::for_wavelength (colour_xyz.rs:22-29). */
void vr_colour_xyz_for_wavelength(double wavelength, double out[3]);
/* mesh::load_obj (src/mesh.rs:74-88): positions/normals parsed as f32 then widened, polygons
 * fan-triangulated; missing normals are zero.  Returns a malloc'ed [n][3][3] pair; free with
 * vr_mesh_free. */
int vr_load_obj(const char* path, uint64_t* triangle_count, double** vertices, double** normals);
void vr_mesh_free(double* vertices, double* normals);

/* AccumulationBuffer::to_image_rgb_u8(&ClampingToneMapper) (accumulation_buffer.rs:38-42,
 * image.rs:166-187, colour_xyz.rs:49-84): XYZ -> linear sRGB (the reference's matrix) ->
 * srgb_gamma (its constants 12.98 / 1.005) -> clamp to [0, 1] -> (v * 255) truncated (NaN -> 0).
 * vr_tone_map_device: `state` = device records (as vr_render_tile_device writes them; only the
 * sums half is read; colour = colour_sum * (1 / weight), 0 where weight is 0), `rgb_out` = device memory
 * (3 bytes per pixel, row-major); enqueued on `stream` (NULL = the null stream) of `device`.
 * vr_tone_map: host XYZ colour buffer (3 f64 per pixel) -> host RGB bytes. */
int vr_tone_map_device(const double* state, uint64_t pixel_count, uint8_t* rgb_out, int device, void* stream);
int vr_tone_map(const double* colour_xyz, uint64_t pixel_count, uint8_t* rgb_out, int device);
/* ImageRgbU8::write_png (image.rs:52-66): 8-bit RGB PNG of `height` rows of `width` pixels
 * (row 0 first).  Host only. */
int vr_write_png(const char* path, const uint8_t* rgb, uint32_t width, uint32_t height);

/* Upper bound on the staging memory one render call may use (16 B per pixel-sample of a launch;
 * 0 = the default, half of the free HBM).  A call whose tile x spp needs more runs in several
 * launches that continue update_pixel in sample order (bit-identical records).  For a GPU shared
 * with other work, and the tests of the pass split.  Not thread-safe against concurrent render
 * calls on the same scene: set it before rendering (ABI 7). */
int vr_scene_set_staging_limit(vr_scene* scene, uint64_t bytes);

/* Test hook (no reference counterpart): every hit on scene object `object` takes the singular-
 * shading-basis path (VR_ERROR_SINGULAR_BASIS, where simple_random_integrator.rs:26-31 panics),
 * which finite geometry cannot reach; -1 turns it off.  Not thread-safe against concurrent render
 * calls on the same scene: set it before rendering (tests/test_gpu_concurrency.py).  ABI 5. */
int vr_debug_set_fault_object(vr_scene* scene, int32_t object);

/* Test hook: launch flags (VR_LAUNCH_NO_CULL / _NO_DIST_CULL / _NO_COOP / _NO_LONE_WALK only) applied to every render
 * call of the scene, including the host-buffer and per-sample record entry points that take no launch
 * flags of their own; 0 turns them off.  Set before rendering, like the fault object (ABI 8). */
int vr_debug_set_launch_flags(vr_scene* scene, uint32_t flags);
/* 1 when a scene with this many triangles and 4-wide nodes renders with the 64-bit-offset kernels
 * (VR_SCENE_WIDE_OFFSETS), else 0.  Host only, no device (ABI 8). */
int vr_scene_needs_wide_offsets(uint64_t triangle_count, uint64_t wide_node_count);

int vr_device_count(void);
const char* vr_last_error(void);
uint32_t vr_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* VANRIJN_AMD_H */

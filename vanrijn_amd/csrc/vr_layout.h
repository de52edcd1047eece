// vr_layout.h -- HBM layout of a flattened scene and the kernel parameter blocks.
//
// Shared by the host side (vr_scene.cpp, vr_capi.cpp) and the gfx950 kernels (vr_render.hip).
// Sizes are chosen for 64-lane waves doing independent per-lane gathers: every record a lane
// reads whole is a multiple of 16 B and 16-B aligned so it is fetched with dwordx4 loads.
#pragma once

#include <stdint.h>

namespace vr {

constexpr int kRecursionLimit = 128;       // camera.rs:69
constexpr int kMaxSpectrumSamples = 64;
constexpr double kBounceBias = 0.0000001;  // simple_random_integrator.rs:42
// VR_LAUNCH_DEFER_TIMES launches a stream may hold before vr_collect_launch_times (3 HIP events each)
constexpr uint32_t kMaxDeferredLaunches = 4096;

// One interior node of a binary BVH, child boxes stored in the parent so a visit tests both
// children with one 128-B record.  box[c] = {min x, max x, min y, max y, min z, max z} of child c
// (its own bounds in the reference tree, bounding_volume_hierarchy.rs:18-28).  child[c] >= 0:
// interior node index; child[c] < 0: leaf holding triangle ~child[c] (leaf size is always 1,
// bounding_volume_hierarchy.rs:57).
struct alignas(128) Node {
    double box[2][6];  // 96 B
    int32_t child[2];  //  8 B
    int32_t pad[6];    // 24 B -> 128 B, one cache line
};
static_assert(sizeof(Node) == 128, "Node must be one 128-B line");

// The traversal tree the render kernel walks: a 4-wide BVH collapsed from the binary traversal
// tree (the reference's closest hit does not depend on the tree's shape), so
// a ray's chain of dependent node fetches is about half as long as in the binary tree.  Child
// boxes are rounded OUTWARD to f32 (each f32 box contains its f64 box); child[c] >= 0: wide node
// index, child[c] < 0 (and != kEmptyChild): leaf holding triangle ~child[c], whose box is the
// triangle's own box; kEmptyChild: unused slot.  A box test is decided from this record unless
// the f32 interval is within its error bound of a tie; then an interior child is descended (a
// superset box: only extra work) and a leaf child's exact f64 test runs on the triangle's own box,
// recomputed from its vertices in the leaf round.
constexpr int32_t kEmptyChild = INT32_MIN;  // ~INT32_MAX: never a triangle (tri_count <= INT32_MAX)
struct alignas(128) Node4 {
    float box[4][6];   // 96 B: {min x, max x, min y, max y, min z, max z} per child
    int32_t child[4];  // 16 B
    int32_t pad[4];    // 16 B -> 128 B, one cache line
};
static_assert(sizeof(Node4) == 128, "Node4 must be one 128-B line");

// Triangle vertices in traversal-BVH leaf order, 80 B for 16-B aligned loads.  `rank` is the
// triangle's scene-wide position in the REFERENCE tree's in-order leaf sequence (tri_base + leaf
// position of the median-split build): equal-distance hits go to the higher rank, as
// closest_intersection's `b` wins ties (bounding_volume_hierarchy.rs:77-92).  The traversal
// tree itself may differ from the reference's (the reference's result does
// not depend on its topology).
struct alignas(16) TriVerts {
    double v[9];
    int64_t rank;
};
static_assert(sizeof(TriVerts) == 80, "TriVerts must be 80 B");

// Shading normals, same order (read once per closest triangle hit).
struct alignas(16) TriNormals {
    double n[9];
    double pad;
};

struct Material {
    int32_t kind;  // 0 Lambertian, 1 Reflective, 2 Phong, 3 smooth transparent dielectric
    int32_t n;     // spectrum sample count (colour; the refractive index for the dielectric)
    double shortest, longest;
    double diffuse, reflection;  // reflection = Phong's specular_strength
    double smoothness;           // Phong exponent
    double samples[kMaxSpectrumSamples];
    // spectrum.rs:64-79's sample wavelengths, (j / (n - 1)) * range + shortest, evaluated on the
    // host with the reference's operations (bit-identical), and (n - 1) / range: the device's
    // intensity lookup (material_intensity) needs one division instead of four
    double knots[kMaxSpectrumSamples];
    double inv_step;
};

// Plane (after Plane::new) or sphere.
struct Prim {
    int32_t kind;      // 0 plane, 1 sphere
    int32_t material;
    int32_t object;    // scene object index
    int32_t position;  // position inside its primitive list
    double vec[3];     // plane normal / sphere centre
    double tan[3];     // plane tangent
    double cot[3];     // plane cotangent
    double scalar;     // plane distance / sphere radius
    // ray-independent products the tests would recompute per ray (same f64 operations, so the
    // same bits): plane: q = normal * distance (plane.rs:57); sphere: centre * centre per
    // component and radius * radius (sphere.rs:48-57)
    double pre[3];
    double scalar2;
};

struct Bvh {
    double root_box[6];  // bounds of the whole tree (tested first, as the reference's root)
    float root_box32[6];  // the same, rounded outward to f32 (the slab32 pre-test)
    int32_t root;        // >= 0 interior node, < 0 leaf ~triangle, INT32_MIN: empty mesh
    int32_t root4;       // the same in the 4-wide tree (>= 0: Node4 index)
    int32_t pad_b;
    int32_t object;      // scene object index
    int32_t tri_base;    // first triangle of this mesh in the global leaf-ordered arrays
    int32_t material;
};

// Device view of a scene (all pointers are device pointers on one GPU).
struct DeviceScene {
    const Node* nodes;     // binary tree (trace / shadow rays)
    const Node4* nodes4;   // 4-wide traversal tree (render kernel)
    const TriVerts* tris;
    const TriNormals* normals;
    const Material* materials;
    const Prim* prims;
    const Bvh* bvhs;
    int32_t prim_count;
    int32_t bvh_count;
    double camera[3];
    double margin;         // distance-cull slack (absolute + relative), see DESIGN.md "Traversal"
    double behind_margin;  // cull of boxes entirely behind the origin
    double extent;         // max |coordinate| of camera and geometry (f32 box-test error bound)
    // integrator: 0 SimpleRandomIntegrator (camera.rs:103), 1 WhittedIntegrator
    // (whitted_integrator.rs:15-87): its ambient spectrum is materials[light_base], light j's
    // spectrum materials[light_base + 1 + j], its direction light_dirs[3j..3j+2]
    int32_t integrator;
    int32_t light_count;
    int32_t light_base;
    int32_t sky_row;       // materials[sky_row]: knots / inv_step of the RGB basis (the sky lookup)
    const double* light_dirs;
};

struct RenderArgs {
    DeviceScene scene;
    uint64_t start_column, start_row, tile_width, tile_height;
    uint64_t width, height;
    uint64_t seed, first_sample;  // absolute index of this pass's sample 0
    uint64_t seed_key;            // mix64(seed ^ salt): the stream key, once per launch
    uint32_t spp;                 // samples in this pass
    uint32_t accumulate;
    uint32_t shade_threshold;     // lanes finished with traversal before the wave shades
    uint32_t chunk;               // samples per work item (one pixel x `chunk` consecutive samples)
    uint32_t phase_a_reps;        // max shade/generate rounds before traversal resumes
    uint32_t tail_samples;        // the launch's last samples go out as single-sample items
    uint32_t grab;                // items a wave takes from the queue per atomic (0: exactly its need)
    uint32_t leaf_threshold;      // leaf round once this many lanes have a pending triangle ...
    uint32_t leaf_stall;          // ... or this many lanes cannot step without one
    uint32_t leaf_few;            // ... or at most this many lanes are still traversing
    // the launch's tail (COOP instantiations): a wave's last 1 to `coop` (4) paths walk their trees
    // with the wave's lanes once each has bounced `coop_bounces` times (coop_step: 1 or 2 owners,
    // lone_walk's whole walks: up to 4); 0: off
    uint32_t coop;
    uint32_t coop_bounces;
    // 1: the tail's walks with nothing pending run whole in lone_walk (0: coop_step only; test hook)
    uint32_t lone_walk;
    uint32_t sort_mask;           // node step's packed child keys: low bits = child index (2^k - 1 > every wide node index)
    // work-item order: 0 sample-major (item = (sample round, block, pixel): the chip's waves in flight
    // cover the whole tile), 1 block-major (item = (block, sample round, pixel): they cover a few
    // blocks, so their camera rays -- and the first hits' tree paths -- are shared)
    uint32_t item_order;
    int32_t fault_object;         // test hook: hits on this object take the singular-basis path (-1: none)
    uint32_t shade_min;           // defer shading until this many lanes have hits (0: never defer)
    uint32_t miss_min;            // defer finishing misses until this many lanes missed (0: never)
    // 1: a path whose throughput and affine term are both 0 ends early (its intensity is 0 for
    // every continuation) -- set only for scenes whose continuations are provably finite
    // (vr_host.cpp shading_finite); 0: traced to the end like the reference, so 0 * NaN stays NaN
    uint32_t early_stop;
    // ImageSampler film constants (camera.rs:24-66): film_w * (1 / width), film_w * 0.5,
    // film_h * (1 / height), film_h * 0.5 -- the kernel's expressions, evaluated once
    double film[4];
    // work-item decode without integer division: 1 / (8x8 blocks per sample round), 1 / (blocks
    // per row), as f64 (a 32-bit quotient from one f64 product is off by at most one, then fixed)
    double rcp_blocks, rcp_bw;
    unsigned long long* queue;    // work-item counter (zeroed before the launch)
    double* staging;              // [pass sample][tile pixel][2] final photon {wavelength, intensity}
    // [tile pixels][4] sums {X, Y, Z, weight}, then [tile pixels][4] compensations {X, Y, Z,
    // weight} (include/vanrijn_amd.h, ABI 7): the cross-GPU reduce adds the first half in place
    double* state;
    void* records;             // vr_sample_record* (record variant) or nullptr
    unsigned long long* counters;  // [kCntCount] (counting variant) or nullptr
    unsigned long long* wg_times;  // counting variant: [blocks][2] s_memrealtime at start / end, or nullptr
    int32_t* error_flag;          // this call's error word (a singular shading basis sets it)
    // per 8x8 pixel block of the tile: 1 when every camera ray through the block provably misses
    // every object (block_cull_kernel), so each of its samples is photon {0, 0}; nullptr: none
    const uint8_t* block_mask;
    // the tile's 8x8 blocks that are NOT culled, in block order (block_compact_kernel), and their
    // count: work items enumerate only these, so culled blocks cost the work queue nothing;
    // nullptr: every block of the tile is live
    const uint32_t* live_blocks;
    const uint32_t* live_count;
    // debug builds only (-DVR_STAGE_GUARD, DESIGN.md section 8 "staging invariant"): beside every
    // staged photon the launch's generation, which the ordered reduce checks before reading it
    // analysis builds only (-DVR_SPLIT_PROBE, DESIGN.md section 6 "the megakernel split"): the render
    // kernel appends every traced ray (6 f64) to probe_rays (probe_count: the next slot; at most
    // probe_n); the TRACE kernel reads probe_n rays from it and writes their closest hits (2 f64
    // each) to probe_hits
    const double* probe_rays;
    double* probe_hits;
    unsigned long long* probe_count;
    uint64_t probe_n;
    uint32_t* stage_tag;  // [pass sample][tile pixel], or nullptr
    uint32_t stage_gen;   // this pass's generation (never 0)
    uint32_t pad_gen;
};

struct TraceArgs {
    DeviceScene scene;
    uint64_t n;
    const double* origins;
    const double* directions;
    void* out;  // vr_hit_record*
};

// counters[] slots of the counting kernel variant
enum Counter : int {
    kCntBoxTests = 0,
    kCntNodeVisits = 1,
    kCntTriangleTests = 2,
    kCntRays = 3,
    kCntShadedTriangles = 4,
    kCntSamples = 5,
    kCntTraversalSlots = 6,  // 64 x wave-level traversal-loop iterations (lane-slot occupancy)
    kCntOuterSlots = 7,      // 64 x wave-level path-loop iterations
    kCntExactBoxes = 8,      // f32 box tests that fell back to the exact f64 test
    kCntCycles = 9,          // 9..14: wave clock cycles per section (diagnostic, VR_COUNTERS_PATH):
                             // shade, refill, camera + begin_ray, node step, leaf round, next BVH + loop
    kCntSections = 15,       // 15..23: wave-level executions of code sections (diagnostic):
                             // leaf test, 2nd leaf test, exact box, shade, camera, begin_ray,
                             // finish, refill, start_bvhs in traversal
    kCntStepHist = 24,       // 24..32: phase-B iterations by the number n of lanes taking a node
                             // step in them: n = 0, then 1-8, 9-16, .., 57-64 (diagnostic, VR_COUNTERS_PATH)
    kCntPrimTests = 33,      // 33..35 (diagnostic, VR_COUNTERS_PATH): wave-level f64 sphere tests run,
                             // their lanes whose f32 pre-test may hit, their active lanes
    kCntCount = 36
};

// Launch wrappers implemented in vr_render.hip (host-callable).
// Which render_kernel instantiation a launch runs (vr_host.cpp enqueue_passes picks, vr_render.hip
// launch_render maps it to the template).
struct LaunchChoice {
    int stack_depth;  // LDS stack entries the scene's traversal needs (class 24 / 32 / 48)
    bool counting;    // the counting variant (VR_LAUNCH_COUNTERS)
    bool recording;   // the per-sample record variant (vr_render_samples)
    bool dark0;       // every material's colour at 0 nm is 0
    int mats;         // material kinds present (bit 0 Lambertian, 1 reflective, 2 Phong / dielectric)
    bool coop;        // the cooperative-tail instantiation (RenderArgs::coop set; never with the above)
    bool big;         // 64-bit node / triangle load offsets (vr_host.cpp needs_big_offsets)
    bool s16;         // 16-bit LDS stack entries (trees below 65,536 wide nodes; timed kernels only)
};
int launch_render(const RenderArgs& args, const LaunchChoice& choice, int grid_limit, void* stream,
                  void* mid_event = nullptr);
// vr_image.hip: records (from_state = 1, RenderArgs::state's layout) or XYZ colour (3 f64) -> sRGB8
// the camera-frustum test of every 8x8 block of a launch's tile into mask (RenderArgs::block_mask)
int launch_block_cull(const RenderArgs& args, uint8_t* mask, void* stream);
// the live (unculled) blocks of `mask` (n blocks) in order into live[], their number into *count
int launch_block_compact(const uint8_t* mask, uint32_t bw, uint32_t bh, bool morton, uint32_t* live, uint32_t* count,
                         void* stream);
int launch_tonemap(const double* src, int from_state, uint64_t npix, uint8_t* rgb, void* stream);
// vr_image.hip: device records (RenderArgs::state's layout) <-> the host AccumulationBuffer's five arrays laid
// out back to back (to_planar = 1: records -> planar, 0: planar -> records; colour is not read;
// 2: records -> colour_sum only, 3 f64 per pixel)
int launch_buffer_convert(const double* src, double* dst, uint64_t npix, int to_planar, void* stream);
// vr_build.hip: one mesh's BVH on the device (same nodes and leaf order as the host build)
int device_build_bvh(const double* verts, const double* norms, uint32_t n, int32_t node_base, int32_t tri_base,
                     Node* nodes, TriVerts* tris, TriNormals* normals, uint64_t* leaf_order, double* root_box,
                     int* levels, void* stream);
// vr_build.hip: the binned-SAH traversal tree of one mesh whose reference-order triangles are on the
// device (root at nodes[0]); the triangles are permuted into its leaf order
int device_build_sah(TriVerts* tris, TriNormals* normals, uint32_t n, int32_t node_base, int32_t tri_base,
                     Node* nodes, double* root_box, int* levels, void* stream);
// vr_build.hip: Node4 / Node4x records from a device-built binary tree and a host-made descriptor
int device_fill_wide(const Node* bin, const int32_t* desc, uint64_t n4, Node4* out4, void* stream);
int launch_trace(const TraceArgs& args, int stack_depth, void* stream);
#ifdef VR_SPLIT_PROBE  // analysis builds (vr_render.hip)
int launch_trace_probe(const RenderArgs& args, int stack_depth, int minw, bool s16, int grid, void* stream);
#endif
const char* device_error_string(int code);

}  // namespace vr

// vr_render.hip -- the MI355X (gfx950) hot path: camera rays, closest-hit BVH traversal,
// ray-triangle / sphere / plane tests, the SimpleRandomIntegrator path loop, Lambertian and
// reflective BSDFs and the Kahan-compensated CIE-XYZ accumulation, in one kernel.
//
// Compiled with -ffp-contract=off: every f64 expression below is written in the operation order
// of the reference's Rust text (which never contracts a*b+c), so hit/miss decisions and bounce
// directions are bit-identical to the CPU restatement in oracle/ (SURVEY.md F5/F6).  The only
// re-association is the forward (iterative) accumulation of path throughput, which changes
// values by O(1e-16) relative and no decision.
//
// Execution model:
//   * persistent waves (3 per SIMD) pull single-sample work items (pixel, sample) from a global
//     queue, 512 items per atomic into a wave-private slice (8 consecutive 8x8 pixel blocks);
//   * each lane keeps its own path state; the wave alternates a shading phase (BSDF, next ray,
//     end of sample + next camera ray) and a traversal phase that steps BVH nodes for every
//     traversing lane until 56 lanes wait to shade;
//   * traversal: per-lane ordered stack walk (LDS stack [depth][thread], node indices only) over
//     a 4-wide tree of 128-B f32 nodes with outward-rounded boxes; a box test too close to call
//     in f32 is re-run exactly in f64 on the 192-B Node4x; leaf triangles are queued (8 per lane,
//     LDS) and tested in f64 in leaf rounds when 2 lanes stall, so the triangle test runs for many
//     lanes at once;
//   * each sample's final photon {wavelength, intensity} goes to a staging buffer;
//     accumulate_kernel turns it into XYZ and folds the samples of a pixel in sample order with
//     the reference's Kahan update_pixel, so the buffers are bit-identical to sequential calls.
#include <hip/hip_runtime.h>

#include <float.h>
#include <stdint.h>
#include <stdlib.h>
#include <type_traits>

#include "../../include/vanrijn_amd.h"
#include "rgb_spectrum_tables.h"
#include "vr_layout.h"
#include "vr_exp_table.h"

#include "vr_device.h"

namespace vr {
namespace dev {

// ----------------------------------------------------------------------------------------------
// Kernels
// ----------------------------------------------------------------------------------------------
__device__ __forceinline__ Ray ray_new(V3 o, V3 d) { return Ray{o, normalize(d)}; }  // mod.rs:41-46

// ----------------------------------------------------------------------------------------------
// Render kernel: persistent waves, lane-level work queue, traversal and shading interleaved.
//
// Work items are (pixel, `chunk` consecutive samples), numbered chunk-major over 8x8 pixel
// blocks; chunk = 1 by default (a pixel whose paths all run to the 128-bounce limit would
// otherwise hold one lane for chunk x 128 bounces: 6.5x on the reflective bench scene).  Lanes
// refill from a wave-private slice of the queue (`grab` items per atomic; one atomic per refill
// cost 35 %).  With whole 16x16 blocks x 256 spp per workgroup, average workgroup concurrency
// was 43 % of the chip's; with the queue it is 98 %.
//
// Inside a wave, each lane's traversal state (node, LDS stack, closest hit, pending leaves)
// stays alive across iterations: the wave steps BVH nodes for all traversing lanes until at
// least `shade_threshold` lanes have finished, then those lanes shade and rejoin (one-ray-per-
// iteration lock-step measured 25 % traversal lane utilisation; this scheme 58 %).
// ----------------------------------------------------------------------------------------------
// Lane masks straight from one v_cmp into a scalar register pair (llvm.amdgcn.icmp): __ballot of a
// bool that already lives in a lane mask is lowered to v_cndmask + v_cmp (two extra VALU per vote,
// on the phase-B loop's every iteration)
__device__ __forceinline__ uint64_t lanes_ieq(int a, int b) { return __builtin_amdgcn_sicmp(a, b, 32); }
__device__ __forceinline__ uint64_t lanes_ine(int a, int b) { return __builtin_amdgcn_sicmp(a, b, 33); }
__device__ __forceinline__ uint64_t lanes_igt(int a, int b) { return __builtin_amdgcn_sicmp(a, b, 38); }
__device__ __forceinline__ uint64_t lanes_ige(int a, int b) { return __builtin_amdgcn_sicmp(a, b, 39); }
__device__ __forceinline__ uint64_t lanes_uge(uint32_t a, uint32_t b) { return __builtin_amdgcn_uicmp(a, b, 35); }
__device__ __forceinline__ uint64_t exec_mask() { return __builtin_amdgcn_read_exec(); }
// set bits of the wave mask m in lanes below this one (two v_mbcnt, no lane-mask registers)
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// Items of one launch: the first spp - tail samples in chunks of `chunk`, then the last `tail`
// samples one per item, so that a path that runs to the recursion limit near the end of the
// launch holds one lane for one path, not for `chunk` of them.
// keeps a wave-uniform 64-bit value in SGPRs
__device__ inline uint64_t uniform64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__host__ __device__ inline uint32_t tail_of(const RenderArgs& a) {
    return a.tail_samples < a.spp ? a.tail_samples : a.spp;
}
__host__ __device__ inline uint64_t chunk_rounds(const RenderArgs& a) {
    const uint32_t bulk = a.spp - tail_of(a);
    return (bulk + a.chunk - 1) / a.chunk;
}
__host__ __device__ inline uint64_t render_items(const RenderArgs& a, uint64_t per_chunk) {
    return per_chunk * (chunk_rounds(a) + tail_of(a));
}

// kRayReady: the lane's next ray (pre.o, pre.d) is set and begin_ray runs once for all such
// lanes at the end of phase A (one inlined copy for bounce and camera rays alike)
//
// Wave-level leaf queue: the leaf triangles a wave's lanes meet go to one FIFO per wave, tagged
// with the lane whose ray met them, and a leaf round hands the oldest 64 to the 64 lanes -- each
// tests one against its owner's ray (fetched by cross-lane permute), and the owners merge their
// results through LDS atomics.  The f64 triangle test then runs with every lane busy; with per-lane
// queues a round tested one triangle per lane that had one (17 of 64).
//
// Wave priority by phase (s_setprio; MI355X_MICROARCH.md: VALU issue is arbitrated by priority,
// then age): a wave stepping BVH nodes or testing leaves -- short, latency-bound bursts ending in
// a dependent load -- wins issue over waves in long f64 shading sequences, so its next load
// leaves sooner.  Measured (A/B): traversal 1 / shading 0: main -1.0 %, C5 -2.0 %; the reverse
// +1.1 %, +3.4 %.
//
// Experiments measured and rejected in rounds 2-3 (the f32 sphere skip, the plane-sign skip, lazy
// shear constants, per-lane leaf queues, rotated vertex loads, the hoisted sphere reciprocal, the
// cooperative tail, the partial child sort, plain staging stores) were removed from the source in
// round 4; their code is kept as a patch (profiles/r04/removed_experiments.patch) and their A/B
// numbers in DESIGN.md.
#ifndef VR_PRIO  // phase A, node step, leaf round (A/B builds: -DVR_PRIO=0,2,1 ...)
#define VR_PRIO 0, 1, 1
#endif
constexpr int kPrio[3] = {VR_PRIO};
constexpr int kPrioA = kPrio[0], kPrioNode = kPrio[1], kPrioLeaf = kPrio[2];
#ifndef VR_WATCHDOG  // debug builds: a wave stuck in phase B prints its lanes' state and stops
#define VR_WATCHDOG 0
#endif
#ifndef VR_NODE_STEPS  // node steps per phase-B iteration (round 6: 2)
#define VR_NODE_STEPS 2
#endif
constexpr int kPend = 8;  // FIFO entries per lane of a wave, on average
constexpr int kWaveList = 64 * kPend;
static_assert((kWaveList & (kWaveList - 1)) == 0, "the wave FIFO is a power-of-two ring");
// Room for a node step's leaves: the wave FIFO can take a step of all 64 lanes (4 leaves each), so
// any one lane may queue more than kPend.  Wave-uniform (q_head / q_tail are).
#define VR_ROOM (q_tail - q_head <= (uint32_t)(kWaveList - 256))

// The kernel argument block, re-read through a pointer the compiler cannot prove unchanged: the
// tree and triangle base pointers become scalar loads at their use.  Held in SGPRs for the whole
// kernel they were spilled to VGPR lanes and cost 8 v_readlane per node step (static count
// 245 -> 34; -1.7 % on the main scene, -2 % on the reflective bench scene).
typedef __attribute__((address_space(4))) const RenderArgs* KArgs;
__device__ __forceinline__ KArgs kargs() {
    KArgs p = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return p;
}
#define VR_NODES4 (kargs()->scene.nodes4)
#define VR_TRIS (kargs()->scene.tris)

enum LaneState : int { kNeedRay = 0, kTraversing = 1, kTraversed = 2, kDone = 3, kRayReady = 4 };

#ifdef VR_COOP_PROF
// VR_CP_DUMP (analysis builds): a tail wave's phase sums into words 8..18 of the context's queue
// buffer, and one record per wave that ran for more than 1 ms (vr_host.cpp prints both)
__device__ void coop_prof_dump(unsigned long long* o, bool coop_on, unsigned lane, const uint64_t* cp_t,
                               const uint32_t* cp_n, uint64_t cp_r0, uint64_t cp_s, uint32_t cp_maxlive) {
    if (coop_on && lane == 0) {
        for (int i = 0; i < 4; ++i) atomicAdd(o + i, (unsigned long long)cp_t[i]);
        for (int i = 0; i < 3; ++i) atomicAdd(o + 4 + i, (unsigned long long)cp_n[i]);
        atomicAdd(o + 7, 1ull);
        atomicMax(o + 8, (unsigned long long)(__builtin_amdgcn_s_memrealtime() - cp_r0));
        atomicAdd(o + 10, (unsigned long long)cp_n[3]);
        atomicAdd(o + 9, (unsigned long long)(__builtin_amdgcn_s_memrealtime() - cp_r0));
    }
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    if (now - cp_s > 100000 && lane == 0) {
        const unsigned long long slot = atomicAdd(o + 11, 1ull);
        if (slot < 1000) {
            unsigned long long* r = o + 16 + 6 * slot;
            r[0] = now - cp_s;
            r[1] = coop_on ? now - cp_r0 : 0;
            r[2] = cp_n[3];
            r[3] = cp_n[2];
            r[4] = cp_maxlive;
            r[5] = cp_s;
        }
    }
}
#endif

// MATS: material kinds present (1 Lambertian, 2 reflective, 3 both); code for absent kinds is
// compiled out, which keeps the reflective BSDF's acos/pow/exp off Lambertian-only scenes.
// WHITTED: the WhittedIntegrator (whitted_integrator.rs:20-87) instead of SimpleRandomIntegrator.
// COOP: the cooperative tail (coop_step below) -- instantiated for the small launches of scenes with
// a reflective material, the only ones whose time is a few trapped paths (vr_host.cpp make_args).
// BIG: 64-bit byte offsets for the node and triangle loads -- scenes whose triangle array reaches 4 GB
// (53.7 M triangles) or whose 4-wide tree has 2^25 nodes (vr_host.cpp needs_big_offsets); every other
// scene's kernels address both arrays with 32-bit offsets from the scalar base (the loads' saddr form)
// TRACE (analysis builds, -DVR_SPLIT_PROBE: DESIGN.md section 6, "the megakernel split"): the same
// kernel as a traversal-only pass over a buffer of rays -- work items are rays (RenderArgs::probe_rays,
// 6 f64 each), phase A stores each closest hit (probe_hits, 2 f64: distance, kind | index << 2 and
// object) instead of shading, and no path state exists, so the register peak is traversal's alone.
// S16: 16-bit LDS stack entries (trees below 65,536 wide nodes): half the stack's LDS, so more
// workgroups fit a CU.
template <int STACK, bool COUNT, bool RECORD, bool DARK0, int MATS = 3, int MINW = 3, bool WHITTED = false,
          bool COOP = false, bool BIG = false, bool TRACE = false, bool S16 = false>
// The scene's small uniform tables (planes / spheres, materials, BVH roots) come in again as
// restrict-qualified arguments: nothing the kernel stores can alias them, so their wave-uniform
// reads compile to scalar loads (the scalar cache) instead of vector loads through L2.
__global__ __launch_bounds__(256, MINW) void render_kernel(RenderArgs A, const Prim* __restrict__ g_prims,
                                                           const Material* __restrict__ g_materials,
                                                           const Bvh* __restrict__ g_bvhs) {
    typedef typename std::conditional<S16, uint16_t, uint32_t>::type StackT;
    __shared__ StackT st_node[STACK * 256];
    // leaf triangles met during traversal wait for a leaf round, in which every lane tests one: the
    // f64 triangle test then runs for many lanes at once instead of for the few that reached a leaf
    // in this step.  Per wave: the FIFO of queued leaves (triangle | exact-box flag, and the owning
    // lane) and, per owner lane, one leaf round's results: entries tested, min distance bits, and
    // (max rank at that distance, its triangle)
    __shared__ int32_t wl_tri[4 * kWaveList];
    __shared__ uint8_t wl_own[4 * kWaveList];
    __shared__ unsigned long long lr_d[256], lr_key[256];  // key: rank << 32 | triangle
    __shared__ uint32_t lr_cnt[256];
    // COOP: an owner's stack column map (coop_step)
    __shared__ uint32_t coop_map[COOP ? 256 : 1];
    const int wbase = (threadIdx.x >> 6) * kWaveList;
    uint32_t q_head = 0, q_tail = 0;  // wave-uniform FIFO positions (mod kWaveList)
    const int tid = threadIdx.x;
    const unsigned lane = __lane_id();
    lr_d[tid] = ~0ull;  // each lane's result slot is only touched by its own wave
    lr_key[tid] = 0;
    lr_cnt[tid] = 0;
    if (COOP) coop_map[tid] = 0;
    DeviceScene S = A.scene;
    S.prims = g_prims;
    S.materials = g_materials;
    S.bvhs = g_bvhs;
    Counts cnt = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t sec[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t step_hist[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // counting variant: lanes per node step
    uint32_t prim_cnt[3] = {0, 0, 0};  // counting variant: sphere tests, their maybe-lanes, active lanes
#ifdef VR_MARKS  // ISA section markers for tools/isa_sections.py (analysis builds only)
#define VR_MARK(name) asm volatile(";@mark " name)
#else
#define VR_MARK(name)
#endif
#define VR_SEC(i) \
    if (COUNT && first_active_lane()) sec[i]++;
    uint64_t cyc[6] = {0, 0, 0, 0, 0, 0}, tprev = COUNT ? __builtin_amdgcn_s_memtime() : 0;
#define VR_STAMP(i)                                           \
    if (COUNT) {                                              \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();     \
        cyc[i] += t_ - tprev;                                 \
        tprev = t_;                                           \
    }
    uint32_t samples_done = 0;
    // The cooperative tail's profile (analysis builds, -DVR_COOP_PROF: where a tail wave's time goes;
    // vr_host.cpp prints the sums after the launch).  One macro family, empty in every other build:
    //   VR_CP(i)        s_memtime since the last stamp into phase i (0 phase A, 1 coop steps, 2 leaf
    //                   rounds, 3 the rest of phase B), in tail waves;
    //   VR_CPN(i, c)    event count i when c (0 lone-walk iterations, 1 leaf rounds, 2 phase A
    //                   entries, 3 lone walks);
    //   VR_CP_PHASE_A() phase A starts;  VR_CP_TAIL(n) the wave's live paths before its tail and the
    //                   tail's start time;  VR_CP_DUMP() the wave's records at its end
#ifdef VR_COOP_PROF
    uint64_t cp_t[4] = {0, 0, 0, 0}, cp_prev = 0;
    uint32_t cp_n[4] = {0, 0, 0, 0};
    uint64_t cp_r0 = 0;  // s_memrealtime (100 MHz) when the wave's tail began
    const uint64_t cp_s = __builtin_amdgcn_s_memrealtime();
    uint32_t cp_maxlive = 0;
#define VR_CP(i)                                              \
    if (coop_on) {                                            \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();     \
        cp_t[i] += t_ - cp_prev;                              \
        cp_prev = t_;                                         \
    }
#define VR_CPN(i, c) \
    if (c) cp_n[i]++;
#define VR_CP_PHASE_A()                          \
    cp_prev = __builtin_amdgcn_s_memtime();      \
    VR_CPN(2, coop_on)
#define VR_CP_TAIL(n)                                                           \
    if (!coop && (n) > (int)cp_maxlive) cp_maxlive = (n);                      \
    if (coop_on && cp_r0 == 0) cp_r0 = __builtin_amdgcn_s_memrealtime();
#define VR_CP_DUMP() coop_prof_dump((unsigned long long*)A.queue + 8, coop_on, lane, cp_t, cp_n, cp_r0, cp_s, cp_maxlive)
#else
#define VR_CP(i)
#define VR_CPN(i, c)
#define VR_CP_PHASE_A()
#define VR_CP_TAIL(n)
#define VR_CP_DUMP()
#endif
    if (COUNT && A.wg_times && tid == 0) A.wg_times[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    const uint32_t bw = (uint32_t)((A.tile_width + 7) / 8), bh = (uint32_t)((A.tile_height + 7) / 8);
    // work items run over the live blocks only (frustum-culled blocks are not in the item space)
    const uint32_t nlive = A.live_blocks ? __builtin_amdgcn_readfirstlane(*A.live_count) : bw * bh;
    const double rcp_live = A.live_blocks ? 1.0 / (double)nlive : A.rcp_blocks;
    const uint64_t per_chunk = (uint64_t)nlive * 64;
    const uint64_t items = render_items(A, per_chunk);
    const uint64_t rounds = chunk_rounds(A);
    const double rcp_R = A.item_order ? 1.0 / (double)(rounds + tail_of(A)) : 0.0;  // block-major decode
    const uint32_t bulk = A.spp - tail_of(A);
    const uint64_t npix = A.tile_width * A.tile_height;
    uint32_t px = 0, py = 0, s_end = 0;
    int state = kNeedRay;  // with s_idx == s_end: needs a work item
    uint32_t s_idx = 0;
    bool coop_on = false;  // COOP: this wave's tail walks its last paths cooperatively (sticky)
    uint64_t w_next = 0, w_end = 0;  // this wave's slice of the queue (grab > 0)
    Rng rng;
    rng.reset(0);
    RayPre pre;
    Ray32 pre32;
    Best best;
    int node = -1, sp = 0, bvh_i = 0, cur_object = 0;
    int np = 0;  // this lane's queued leaf triangles not yet tested
    // f32 forms of the cull thresholds, widened by the ray's slab margin E (vr_device.h Ray32):
    // cull_far >= bound + margin + E (rounded up), cull_behind <= -behind_margin - E (rounded down;
    // -inf when behind-culling is off), compared with the slab values lo / hi as computed
    float cull_far = INFINITY, cull_behind = -INFINITY;
    int depth = -1, bounces = 0, flags = 0;
    double lambda = 0.0, T = 1.0, Acc = 0.0, T0 = 1.0, Acc0 = 0.0, b0 = 0.0, wo_y = 0.0;
    double Wa = 0.0, Wb = 0.0;  // Whitted: the pending continuation's throughput and constant

    // BVH cull: subtree entirely beyond the closest hit (+margin) or behind the origin
    auto culled = [&](double tlo, double thi) {
        const double bound = best.kind ? best.d : INFINITY;
        if (tlo > bound + S.margin * (1.0 + fabs(bound))) return true;
        return pre.behind_ok() && thi < -S.behind_margin;
    };
    auto set_cull_far = [&]() {
        const double bound = best.kind ? best.d : INFINITY;
        cull_far = round_away_f32(bound + S.margin * (1.0 + fabs(bound)) + margin_of(pre32));
    };
    // closest_intersection's rule for a triangle hit of the current BVH at distance d, reference rank
    // rk: the smaller distance; at equal distances the later in-order leaf (higher rank) within the
    // BVH, the earlier object across objects (sampler.rs min_by).  Branch-free selects on the rank
    // kept in `best` (round 4: the nested branch form with a global load of the best triangle's rank
    // was miscompiled in some builds -- a tie's new triangle index lost to the old one -- and the
    // load was a dependent global access inside a divergent branch anyway)
    // the triangle record of leaf link ~tri and the 4-wide node `n`
    auto tri_at = [&](int tri) -> const TriVerts* {
        if (BIG) return VR_TRIS + (uint32_t)tri;
        return (const TriVerts*)((const char*)VR_TRIS + (uint32_t)tri * (uint32_t)sizeof(TriVerts));
    };
    auto node_at = [&](int n) -> const Node4& {
        if (BIG) return VR_NODES4[(uint32_t)n];
        return *(const Node4*)((const char*)VR_NODES4 + ((uint32_t)n << 7));
    };
    auto takes_hit = [&](double d, uint32_t rk) {
        const bool closer = !best.kind | (d < best.d);
        const bool tie = (d == best.d) & ((best.object == cur_object) ? (rk > best.rank) : (cur_object < best.object));
        return closer | tie;
    };
    // a queued leaf: its triangle index, bit 31 set when the leaf's f32 box test was too close to
    // call -- then the exact f64 line test on the triangle's own box (BoundingBox::from_points of
    // its vertices, triangle.rs:101-105: per axis fmin / fmax in vertex order, the host build's
    // leaf box bit for bit) decides whether the reference reaches the triangle at all
    auto test_tri = [&](int e) {
        const int tri = e & 0x7fffffff;
        const TriVerts tv = load_tri(tri_at(tri));
        if (e < 0) {
            VR_SEC(2);
            VR_MARK("exact_box");
            if (COUNT) cnt.exact_boxes++;
            double bb[6], lo, hi;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                bb[2 * a] = fmin(fmin(tv.v[a], tv.v[3 + a]), tv.v[6 + a]);
                bb[2 * a + 1] = fmax(fmax(tv.v[a], tv.v[3 + a]), tv.v[6 + a]);
            }
            if (!slab(bb, pre, lo, hi)) return;
        }
        if (COUNT) cnt.tri_tests++;
        double b[3];
        const double d = triangle_distance(tv, pre, b);
        if (d < 0.0) return;
        const uint32_t rk = (uint32_t)tv.rank;
        if (takes_hit(d, rk)) {
            best.d = d;
            best.kind = kTri;
            best.index = tri;
            best.rank = rk;
            best.object = cur_object;
            set_cull_far();
        }
    };
    // One leaf round over the n (<= 64) oldest entries of the wave FIFO: lane i tests entry i
    // against its owner's ray.  Per owner, the round's candidate is the minimum distance and, among
    // equal distances, the highest reference rank (LDS atomics; one wave's LDS operations execute
    // in order): applied to `best` with test_tri's rule it gives what testing the entries one by
    // one in any order gives (closest_intersection keeps the later leaf on ties, sampler.rs keeps
    // the earlier object).  Called with the whole wave active.
    auto leaf_round = [&](uint32_t n) {
        const bool mine = lane < n;
        int e = 0;
        uint32_t owner = lane;
        if (mine) {
            const uint32_t pos = (q_head + lane) & (kWaveList - 1);
            e = wl_tri[wbase + pos];
            owner = wl_own[wbase + pos];
        }
        RayPre op;  // the owner's ray
        op.o.x = __shfl(pre.o.x, (int)owner);
        op.o.y = __shfl(pre.o.y, (int)owner);
        op.o.z = __shfl(pre.o.z, (int)owner);
        op.sx = __shfl(pre.sx, (int)owner);
        op.sy = __shfl(pre.sy, (int)owner);
        op.pdz = __shfl(pre.pdz, (int)owner);
        op.flags = __shfl(pre.flags, (int)owner);
        const int oslot = (tid & ~63) + (int)owner;
        double d = -1.0;
        uint32_t rank = 0;
        const int tri = e & 0x7fffffff;
        // The exact box test decides only where the triangle test hits: a leaf whose triangle
        // misses adds nothing whichever way its box test goes (bvh.rs:77-120 tests the triangle only
        // inside a hit box), so the reference's box decision is taken after the triangle test and
        // only for hitting entries -- the wave runs the six f64 divisions only when such an entry
        // exists, not whenever an entry's f32 box test was too close to call.  The counting variant
        // tests every flagged box, so its counters stay the reference's.
        TriVerts tv;
        if (mine) {
            tv = load_tri(tri_at(tri));
            double b[3];
            d = triangle_distance(tv, op, b);  // needs the owner's shear constants, not its direction
            rank = (uint32_t)tv.rank;
            if (COUNT && e >= 0) cnt.tri_tests++;
        }
        // lanes with an entry (lane < n) whose box was too close to call (e < 0) and whose triangle
        // hits (d >= 0), as compares into lane masks
        const uint64_t flagged = __builtin_amdgcn_uicmp(lane, n, 36 /* ult */) & lanes_igt(0, e);
        if (COUNT ? flagged : (flagged & __builtin_amdgcn_fcmp(d, 0.0, 3 /* oge */))) {
            op.d.x = __shfl(pre.d.x, (int)owner);
            op.d.y = __shfl(pre.d.y, (int)owner);
            op.d.z = __shfl(pre.d.z, (int)owner);
            if (mine && e < 0 && (COUNT || d >= 0.0)) {  // the leaf's f32 box test was too close to call
                VR_SEC(2);
                VR_MARK("exact_box");
                if (COUNT) cnt.exact_boxes++;
                double bb[6], lo, hi;
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    bb[2 * a] = fmin(fmin(tv.v[a], tv.v[3 + a]), tv.v[6 + a]);
                    bb[2 * a + 1] = fmax(fmax(tv.v[a], tv.v[3 + a]), tv.v[6 + a]);
                }
                const bool reach = slab(bb, op, lo, hi);
                if (COUNT && reach) cnt.tri_tests++;
                if (!reach) d = -1.0;
            }
        }
        if (mine) atomicAdd(&lr_cnt[oslot], 1u);
        const bool hit = mine && d >= 0.0;
        const unsigned long long bits = (unsigned long long)__double_as_longlong(d);
        if (hit) atomicMin(&lr_d[oslot], bits);
        // at the minimum distance the highest rank wins; its triangle rides in the low half
        if (hit && lr_d[oslot] == bits) atomicMax(&lr_key[oslot], ((unsigned long long)rank << 32) | (uint32_t)tri);
        // owners: fold the round's candidate into the closest hit
        const uint32_t got = lr_cnt[tid];
        if (got) {
            np -= (int)got;
            const unsigned long long db = lr_d[tid];
            if (db != ~0ull) {
                const double dd = __longlong_as_double((long long)db);
                const unsigned long long key = lr_key[tid];
                const uint32_t rk = (uint32_t)(key >> 32);
                if (takes_hit(dd, rk)) {
                    best.d = dd;
                    best.kind = kTri;
                    best.index = (int)(uint32_t)key;
                    best.rank = rk;
                    best.object = cur_object;
                    set_cull_far();
                }
            }
            lr_cnt[tid] = 0;
            lr_d[tid] = ~0ull;
            lr_key[tid] = 0;
        }
    };
    // next BVH (from bvh_i) with work; false when the ray is fully traced
    auto start_bvhs = [&]() {
        for (; bvh_i < S.bvh_count; ++bvh_i) {
            const Bvh& bvh = S.bvhs[bvh_i];
            if (bvh.root4 == INT32_MIN) continue;
            cur_object = bvh.object;
            if (COUNT) cnt.box_tests++;
            float flo, fhi;
            const int rr = slab32(bvh.root_box32, pre32, flo, fhi);
            if (rr == 0) continue;
            if (rr == 1) {
                if (flo > cull_far || fhi < cull_behind) continue;
            } else {
                double lo, hi;
                if (!slab(bvh.root_box, pre, lo, hi) || culled(lo, hi)) continue;
            }
            if (bvh.root4 < 0) {  // a one-triangle BVH
                test_tri(~bvh.root4);
                continue;
            }
            node = bvh.root4;
            sp = 0;
            return true;
        }
        return false;
    };
    // the lane's next ray, already in pre.o / pre.d (directions normalised; the next ray is kept
    // there, not in registers of its own that would stay live through the traversal phase):
    // primitive lists first, then the BVHs
    auto begin_ray = [&]() {
#ifdef VR_SPLIT_PROBE  // analysis builds: every traced ray's (origin, direction) into probe_rays
        if (!TRACE && A.probe_rays) {
            const uint64_t m = exec_mask();
            const unsigned leader = (unsigned)__builtin_ctzll(m);
            unsigned long long b = 0;
            if (lane == leader) b = atomicAdd(A.probe_count, (unsigned long long)__popcll(m));
            const uint64_t slot = uniform64(__shfl(b, (int)leader)) + lanes_below(m);
            if (slot < A.probe_n) {
                double* r = const_cast<double*>(A.probe_rays) + 6 * slot;
                r[0] = pre.o.x; r[1] = pre.o.y; r[2] = pre.o.z;
                r[3] = pre.d.x; r[4] = pre.d.y; r[5] = pre.d.z;
            }
        }
#endif
        pre = prepare(Ray{pre.o, pre.d});
        pre32 = prepare32(pre, S.extent);
        if (COUNT) cnt.rays++;
        best.kind = kNone;
        best.d = 0.0;
        best.index = -1;
        best.rank = 0;
        best.object = 0x7fffffff;
        VR_MARK("br_prims");
        for (int i = 0; i < S.prim_count; ++i) {
            const Prim& pr = S.prims[i];
            double dd;
            bool ok;
            if (pr.kind == 0) {
                VR_MARK("br_plane");
                ok = plane_distance(pr, pre, dd);
            } else {
                VR_MARK("br_sphere");
                // the f64 test is skipped only when, for every lane, the line clearly misses the
                // sphere or the sphere lies behind the origin or beyond the lane's best distance
                // (camera rays of a wave are coherent; so are many bounce rays)
                const uint64_t maybe_lanes = sphere_maybe32_lanes(pr, pre);
                if (maybe_lanes == 0) continue;
                if (COUNT) {
                    const int act = __popcll(exec_mask());
                    if (first_active_lane()) {
                        prim_cnt[0]++;
                        prim_cnt[1] += __popcll(maybe_lanes);
                        prim_cnt[2] += act;
                    }
                }
                {
                    const double a1 = sphere_a(pre.d);
                    dd = sphere_distance(pr, pre, a1, 1.0 / (2.0 * a1));
                }
                ok = dd >= 0.0;
            }
            if (ok && (!best.kind || dd < best.d)) {  // min_by keeps the first of equals
                best.d = dd;
                best.kind = kPrim;
                best.index = i;
                best.object = pr.object;
            }
        }
        VR_MARK("br_bvhs");
        set_cull_far();
        if (pre.behind_ok()) {
            cull_behind = round_away_f32(-S.behind_margin - margin_of(pre32));
        } else {
            cull_behind = -INFINITY;
        }
        bvh_i = 0;
        node = -1;
        state = start_bvhs() ? kTraversing : kTraversed;
    };
    // the sample's final photon goes to the staging buffer; accumulate_kernel turns it into XYZ
    // (ColourXyz::from_photon of photon.scale_intensity(360)) and the Kahan sums.  finish() only
    // notes the photon; phase A stores it at one place after shading (store_photon), so a wave whose
    // lanes end their samples in different ways (camera miss, sky, recursion limit, early stop)
    // runs the staging address arithmetic once, not once per way
    bool fin = false;
    double fin_wl = 0.0, fin_I = 0.0;
    auto finish = [&](double wl, double I) {
        fin = true;
        fin_wl = wl;
        fin_I = I;
    };
    auto store_photon = [&](double wl, double I) {
        VR_SEC(6);
        VR_MARK("finish");
        double* out = A.staging + ((uint64_t)s_idx * npix + (uint64_t)py * A.tile_width + px) * 2;
        // streamed once to HBM and read once by the reduce: non-temporal, so the 16 B per sample
        // (4.3 GB per 1024^2 x 256 frame) do not evict the BVH and triangles from L2 and MALL
        __builtin_nontemporal_store(wl, &out[0]);
        __builtin_nontemporal_store(I, &out[1]);
#ifdef VR_STAGE_GUARD  // debug builds: this slot now holds this pass's photon
        A.stage_tag[(uint64_t)s_idx * npix + (uint64_t)py * A.tile_width + px] = A.stage_gen;
#endif
        if (RECORD) {
            const double Is = I * 360.0;
            const V3 c = xyz_for_wavelength(wl);
            vr_sample_record* rec =
                (vr_sample_record*)A.records + (((uint64_t)py * A.tile_width + px) * A.spp + s_idx);  // single pass
            rec->wavelength = wl;
            rec->intensity = I;
            rec->xyz[0] = c.x * Is;
            rec->xyz[1] = c.y * Is;
            rec->xyz[2] = c.z * Is;
            rec->bounces = bounces;
            rec->flags = flags;
        }
        if (COUNT) samples_done++;
        ++s_idx;
        state = kNeedRay;
    };
    // one level of SimpleRandomIntegrator::integrate (simple_random_integrator.rs:20-53) at the
    // closest hit, forward form: returns true when a bounce ray was started
    auto shade = [&]() {
        VR_SEC(3);
        VR_MARK("shade");
        HitInfo h;
        hit_info(S, best, pre, h);
        if (COUNT && best.kind == kTri) cnt.shaded++;
        // world_to_bsdf = rows(tangent, cotangent, normal) (algebra_utils.rs:3-5); its
        // determinant via the first-row minors (mat3.rs:106-109)
        const double det = h.tangent.x * (h.cotangent.y * h.normal.z - h.cotangent.z * h.normal.y) -
                           h.tangent.y * (h.cotangent.x * h.normal.z - h.cotangent.z * h.normal.x) +
                           h.tangent.z * (h.cotangent.x * h.normal.y - h.cotangent.y * h.normal.x);
        // try_inverse() == None: the reference panics ("Expected matrix to be invertable."); the
        // fault_object test hook takes this path for hits on one object (DESIGN.md "Errors")
        if (det == 0.0 || best.object == A.fault_object) {
            flags |= 4;
            atomicOr(A.error_flag, 1);
            finish(0.0, 0.0);
            return;
        }
        const V3 w_i = mk(dot(h.tangent, h.retro), dot(h.cotangent, h.retro), dot(h.normal, h.retro));
        const Material* mat = &S.materials[h.material];
        if constexpr (WHITTED) {
            // light terms, in order (fold from the camera photon's intensity 0): a shadow ray per
            // light; blocked -> the ambient spectrum, else bsdf(W retro, W dir, light(lambda) |dir.n|)
            double C = 0.0;
            for (int j = 0; j < S.light_count; ++j) {
                const V3 ldir = ldv(S.light_dirs + 3 * j);
                const V3 d1 = normalize(ldir);
                const RayPre sp = prepare(Ray{add(h.loc, scl(d1, kBounceBias)), normalize_n1(d1)});
                double term;
                if (any_hit<STACK>(S, sp, st_node, tid)) {
                    term = material_intensity(&S.materials[S.light_base], lambda);
                } else {
                    const V3 wl = mk(dot(h.tangent, ldir), dot(h.cotangent, ldir), dot(h.normal, ldir));
                    const double I = material_intensity(&S.materials[S.light_base + 1 + j], lambda) * fabs(dot(ldir, h.normal));
                    double ba, bb;
                    bsdf_affine(mat, w_i, wl, lambda, ba, bb);
                    term = ba * I + bb;
                }
                C = C + term;
            }
            Acc = Acc + T * C;
            if (depth >= kRecursionLimit) {  // recursion_limit 0: the continuation contributes 0
                flags |= 2;
                finish(lambda, Acc);
                return;
            }
        }
        V3 w_o;
        double pdf;
        // material kind: compiled in for the kinds the scene has (MATS 1: Lambertian only,
        // 2: reflective only, 3: any of Lambertian / reflective / Phong / dielectric)
        const int kind = MATS == 1 ? 0 : (MATS == 2 ? 1 : mat->kind);
        Fresnel fr;  // dielectric only
        if (kind == 1) {  // reflective_material.rs:42-47
            w_o = mk(-w_i.x, -w_i.y, w_i.z);
            pdf = 1.0;
        } else if (MATS == 3 && kind == 2) {  // Phong: Material::sample's default (materials/mod.rs:28-33)
            w_o = cosine_weighted_hemisphere(rng);
            pdf = cosine_weighted_pdf(w_o);
        } else if (MATS == 3 && kind == 3) {  // smooth_transparent_dialectric.rs:97-114
            fr = dielectric_fresnel(mat, w_i, lambda);
            pdf = 0.5;
            if (fr.T <= 0.0000000001) w_o = fr.rdir;
            else if (fr.R <= 0.0000000001 || rng.boolean()) w_o = fr.tdir;
            else w_o = fr.rdir;
        } else {  // lambertian_material.rs:36-59: rejection sampling on Open01 pairs
            double x = 2.0 * rng.open01() - 1.0;
            double y = 2.0 * rng.open01() - 1.0;
            while (dot(mk(x, y, 0.0), mk(x, y, 0.0)) > 1.0) {
                x = 2.0 * rng.open01() - 1.0;
                y = 2.0 * rng.open01() - 1.0;
            }
            const double z = fmax(sqrt(1.0 - x * x - y * y), 0.0);
            const V3 w = mk(x, y, z);
            const double cos_theta = dot(w, mk(0.0, 0.0, 1.0));
            const double sin_theta = sqrt(1.0 - cos_theta * cos_theta);
            w_o = normalize_n1(w);  // |w|^2 = x^2 + y^2 + (1 - x^2 - y^2): 1 within a few spacings
            pdf = (cos_theta * sin_theta) / 3.14159265358979323846;
        }
        // bsdf_to_world = cofactor(M)^T * det (mat3.rs:111-118), applied to w_o by rows
        V3 wo_world;
        {
            const double m00 = h.tangent.x, m01 = h.tangent.y, m02 = h.tangent.z;
            const double m10 = h.cotangent.x, m11 = h.cotangent.y, m12 = h.cotangent.z;
            const double m20 = h.normal.x, m21 = h.normal.y, m22 = h.normal.z;
            const V3 inv0 = mk((1.0 * (m11 * m22 - m12 * m21)) * det, (-1.0 * (m01 * m22 - m02 * m21)) * det,
                               (1.0 * (m01 * m12 - m02 * m11)) * det);
            wo_world.x = dot(inv0, w_o);
            const V3 inv1 = mk((-1.0 * (m10 * m22 - m12 * m20)) * det, (1.0 * (m00 * m22 - m02 * m20)) * det,
                               (-1.0 * (m00 * m12 - m02 * m10)) * det);
            wo_world.y = dot(inv1, w_o);
            const V3 inv2 = mk((1.0 * (m10 * m21 - m11 * m20)) * det, (-1.0 * (m00 * m21 - m01 * m20)) * det,
                               (1.0 * (m00 * m11 - m01 * m10)) * det);
            wo_world.z = dot(inv2, w_o);
        }
        const double cosf = fabs(dot(wo_world, h.normal));
        if constexpr (WHITTED) {
            // continuation: bsdf(W retro, dir, L_next) |dir.n|, applied when its ray hits
            double ba, bb;
            bsdf_affine(mat, w_i, w_o, lambda, ba, bb);
            Wa = (T * ba) * cosf;
            Wb = (T * bb) * cosf;
            const V3 d1 = normalize_n1(wo_world);  // an orthonormal basis applied to a unit vector
            ++bounces;
            pre.o = add(h.loc, scl(d1, kBounceBias));  // the next ray (state kRayReady)
            pre.d = normalize_n1(d1);
            state = kRayReady;
            return;
        }
        const double c_l = material_intensity(mat, lambda);
        const double c_0 = DARK0 ? 0.0 : material_intensity(mat, 0.0);
        double a, a0, bterm;
        if (kind == 1) {  // reflective_material.rs:17-39
            if (w_i.z <= 0.0 || w_o.z <= 0.0) {
                a = 0.0; a0 = 0.0; bterm = 0.0;
            } else {
                const V3 refl = mk(-w_o.x, -w_o.y, w_o.z);
                double cth = dot(w_i, refl);
                cth = cth < 0.0 ? 0.0 : (cth > 1.0 ? 1.0 : cth);
                const double theta = acos(fabs(cth));
                const double sigma = 0.05, two = 2.0;
                const double f = mat->reflection * exp(-(pow(theta, two)) / (two * sigma * sigma));
                a = (((pdf * cosf) * c_l) * mat->diffuse) * (1.0 - f);
                a0 = (((pdf * cosf) * c_0) * mat->diffuse) * (1.0 - f);
                bterm = f;
            }
        } else if (MATS == 3 && kind == 2) {  // phong_material.rs:17-36: diffuse + specular lobe
            if (w_i.z < 0.0 || w_o.z < 0.0) {
                a = 0.0; a0 = 0.0; bterm = 0.0;
            } else {
                const V3 refl = mk(-w_i.x, -w_i.y, w_i.z);
                a = ((pdf * cosf) * c_l) * mat->diffuse;
                a0 = ((pdf * cosf) * c_0) * mat->diffuse;
                bterm = pow(fabs(dot(w_o, refl)), mat->smoothness) * (mat->reflection / dot(w_i, mk(0.0, 0.0, 1.0)));
            }
        } else if (MATS == 3 && kind == 3) {  // smooth_transparent_dialectric.rs:79-95
            a = (pdf * cosf) * dielectric_strength(fr, w_o);
            a0 = DARK0 ? 0.0 : (pdf * cosf) * dielectric_strength(dielectric_fresnel(mat, w_i, 0.0), w_o);
            bterm = 0.0;
        } else {  // lambertian_material.rs:27-34
            a = ((pdf * cosf) * c_l) * mat->diffuse;
            a0 = ((pdf * cosf) * c_0) * mat->diffuse;
            bterm = 0.0;
        }
        if (depth == 0) b0 = bterm;
        Acc = Acc + T * bterm;
        T = T * a;
        if (!DARK0) {
            Acc0 = Acc0 + T0 * bterm;
            T0 = T0 * a0;
        }
        // A path whose every continuation yields intensity 0 stops here -- only in scenes the host
        // proved NaN-free (A.early_stop: every mesh triangle's shading basis is finite for any
        // barycentric point, no Phong / dielectric): the reference keeps recursing and returns
        // inner x 0, which is NaN when a later bounce is (simple_random_integrator.rs:39-53).
        const bool zero_tail = DARK0 ? (b0 == 0.0) : (T0 == 0.0 && Acc0 == 0.0);
        if (!RECORD && A.early_stop && T == 0.0 && Acc == 0.0 && zero_tail) {
            finish(lambda, 0.0);  // every continuation yields intensity 0
            return;
        }
        // Ray::new(location, w_o).bias(1e-7): normalise, step, normalise again (mod.rs:41-61)
        wo_y = wo_world.y;
        const V3 d1 = normalize_n1(wo_world);  // an orthonormal basis applied to a unit vector
        ++bounces;
        pre.o = add(h.loc, scl(d1, kBounceBias));  // the next ray (state kRayReady)
        pre.d = normalize_n1(d1);
        state = kRayReady;
    };

    // The launch's tail (COOP instantiations): the queue is exhausted and one or two paths are left
    // in the wave -- in a small frame of a scene with mirrors, paths trapped between facets run to
    // the 128-bounce recursion limit and set the frame's time (C1, benches/simple_scene.rs: 25 of
    // its 3,072 waves hold one or two and end at 3.5-6.4 ms, the others by 1.1 ms).  Their walks are
    // spread over the wave's lanes: with one owner every lane works for it, with two the lower half
    // of the lanes works for the lower owner and the upper half for the other.  Each step takes the
    // owner's current node and up to (workers - 1) entries from the top of its stack, one per worker,
    // tests them against the owner's ray, pushes the hit interior children back and queues the hit
    // leaves for the owner.  An owner's stack spans extra lane columns of the wave (the other lanes
    // are done): with one owner from the start, the next columns in turn; once two owners have shared
    // the wave (coop_map, sticky for the rest of the launch), each owner keeps its own column plus the
    // lanes of its half other than the two owners', so the map never changes under an owner whose
    // partner finishes first.  Culling and the order-independent leaf rounds keep the closest hit and
    // its tie rule: only the visiting order changes.  Called with the whole wave
    // active; `live` holds the one or two live lanes.
    // the LDS word of virtual stack entry v of owner o whose column map is om (coop_map)
    auto coop_vaddr = [&](int o, uint32_t om, int v) {
        const int j = v / STACK, og = (int)(om & 3) - 1, op = (int)(om >> 8);
        int col;
        if (j == 0) {
            col = o;
        } else if (og < 0) {
            col = (o + j) & 63;
        } else {  // the (j-1)-th lane of half og that is neither owner
            const int s1 = o < op ? o : op, s2 = o < op ? op : o, lo = og * 32;
            col = lo + j - 1;
            if (s1 >= lo && s1 < lo + 32 && col >= s1) ++col;
            if (s2 >= lo && s2 < lo + 32 && col >= s2) ++col;
        }
        return (v % STACK) * 256 + (tid & ~63) + col;
    };
    auto coop_step = [&](const uint64_t live) {
        uint32_t lmask = 0;
        int32_t lent[4];
        const int oa = (int)__builtin_ctzll(live);         // lower owner
        const int ob = (int)(63 - __builtin_clzll(live));  // upper owner (== oa: one owner)
        const bool two = oa != ob;
        uint32_t* cmap = &coop_map[tid & ~63];  // per lane: 0 (full map), or 1 + half | partner << 8
        if (two && cmap[oa] == 0) {
            if ((int)lane == oa) cmap[oa] = 1u | ((uint32_t)ob << 8);
            if ((int)lane == ob) cmap[ob] = 2u | ((uint32_t)oa << 8);
        }
        // this lane works for its half's owner (two owners) or the one owner
        const bool upper = two && lane >= 32;
        const int owner = upper ? ob : oa;
        const int gbase = upper ? 32 : 0, gsize = two ? 32 : 64;
        const uint64_t gmask = two ? (upper ? 0xFFFFFFFF00000000ull : 0xFFFFFFFFull) : ~0ull;
        const int r = (int)lane - gbase;  // worker rank
        const uint32_t om = cmap[owner];  // the owner's column map
        const int o_sp = __shfl(sp, owner);
        const int o_node = __shfl(node, owner);
        const bool o_trav = __shfl(state == kTraversing ? 1 : 0, owner) != 0;
        const int have = o_trav ? (o_node >= 0 ? 1 : 0) + o_sp : 0;
        // the owner's stack capacity: every column of the wave, or its own plus 30 of its half
        const int cap = ((om & 3) == 0 ? 64 : 31) * STACK;
        // entries taken this step: at most one per worker, and at most what keeps 150 entries of
        // headroom (a step adds at most 3 net per entry taken; a depth-first walk from a near-full
        // stack needs at most 3 per level below)
        int t = have < gsize ? have : gsize;
        const int room = (cap - 150 - have) / 3;
        if (t > room) t = room < 1 ? (have > 0 ? 1 : 0) : room;
        const bool work = t > 0 && VR_ROOM;  // uniform per half
        uint32_t im = 0;                     // hit interior children
        int c[4] = {0, 0, 0, 0};
        int pos = o_sp;
        // the owner's ray and cull bounds, permuted with the whole wave active: `work` differs between
        // the halves, and the upper half's owner may be a lane of the lower half (ds_bpermute reads 0
        // from a source lane outside exec)
        Ray32 ry;
        ry.ox = __shfl(pre32.ox, owner);
        ry.oy = __shfl(pre32.oy, owner);
        ry.oz = __shfl(pre32.oz, owner);
        ry.ix = __shfl(pre32.ix, owner);
        ry.iy = __shfl(pre32.iy, owner);
        ry.iz = __shfl(pre32.iz, owner);
        ry.nx = __shfl(pre32.nx, owner);
        ry.ny = __shfl(pre32.ny, owner);
        ry.nz = __shfl(pre32.nz, owner);
        ry.e2 = __shfl(pre32.e2, owner);
        const float cf = __shfl(cull_far, owner);
        const float cb = __shfl(cull_behind, owner);
        if (work) {
            VR_MARK("coop_step");
            const int first_stack = o_node >= 0 ? 1 : 0;  // worker 0 takes the current node
            int my = -1;
            if (r < t) my = (r < first_stack) ? o_node : (int)st_node[coop_vaddr(owner, om, o_sp - 1 - (r - first_stack))];
            pos = o_sp - (t - first_stack);  // stack entries left below the taken ones
            if (my >= 0) {
                const Node4& nd = node_at(my);
                if (COUNT) cnt.node_visits++;
                uint32_t xm = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    c[k] = nd.child[k];
                    float f, g;
                    bool maybe, sure;
                    slab32_flags(nd.box[k], ry, f, g, maybe, sure);
                    const bool lv = c[k] != kEmptyChild;
                    if (COUNT && lv) cnt.box_tests++;
                    const bool pass = lv && maybe && !(f > cf || g < cb);
                    xm |= (pass && !sure) ? 1u << k : 0u;
                    im |= (pass && c[k] >= 0) ? 1u << k : 0u;
                    lmask |= (pass && c[k] < 0) ? 1u << k : 0u;
                    lent[k] = (~c[k]) | (((xm >> k) & 1u) ? INT32_MIN : 0);
                }
            }
        }
        // interior hits onto the owner's stack, in (child slot, worker) order
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool ih = (im >> k) & 1u;
            const uint64_t m = __ballot(ih) & gmask;
            if (ih) st_node[coop_vaddr(owner, om, pos + (int)lanes_below(m))] = (uint32_t)c[k];
            pos += (int)__popcll(m);
        }
        // each owner takes its next node, the top of its stack: its workers' pos and work flag
        // (uniform over its half) by permute from the half's first lane
        const int lead = (two && (int)lane == ob) ? 32 : 0;
        const int npos = __shfl(pos, lead);
        const bool nwork = __shfl(work ? 1 : 0, lead) != 0;
        const bool is_owner = ((live >> lane) & 1ull) != 0;
        if (is_owner && nwork) {
            sp = npos;
            if (sp > 0) {
                --sp;
                node = (int)st_node[coop_vaddr((int)lane, cmap[lane], sp)];
            } else {
                node = -1;
            }
        }
        // the hit leaves, queued for their owners in (child slot, lane) order
        const uint64_t own_mask = two ? ((int)lane == ob ? 0xFFFFFFFF00000000ull : 0xFFFFFFFFull) : ~0ull;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool lh = (lmask >> k) & 1u;
            const uint64_t m = __ballot(lh);
            if (lh) {
                const uint32_t qp = (q_tail + (uint32_t)lanes_below(m)) & (kWaveList - 1);
                wl_tri[wbase + qp] = lent[k];
                wl_own[wbase + qp] = (uint8_t)owner;
            }
            q_tail += (uint32_t)__popcll(m);
            if (is_owner) np += (int)__popcll(m & own_mask);
        }
        q_tail = __builtin_amdgcn_readfirstlane(q_tail);
    };
    // The cooperative tail's walks with nothing pending (no stack entries, no queued leaves, an empty
    // wave FIFO) for the one to four traversing paths `own` of a wave whose other lanes are done: the
    // whole rest of each path's walk of its current BVH in one call.  With one owner every lane
    // works for it; with two the lower half works for the lower owner and the upper half for the
    // other, with three or four each quarter of the wave for one of them (round 6: C1 frames whose
    // waves kept three trapped mirror paths took 3.9-5.3 ms against ~1.55 ms, profiles/r06/split/
    // c1_frames.json), all walks at once.  An owner's frontier of nodes to visit is a LIFO over its
    // group's columns of the wave's stack words; each iteration pops up to one node per four workers, each
    // worker tests one child box against the owner's ray, the hit interior children are pushed and
    // the hit leaves tested at once, one per worker.  The round's candidate (minimum distance, then the
    // highest reference rank) is merged with takes_hit's rule, as in leaf_round, so each path gets
    // what its per-lane walk finds: only the visiting order differs.  Against coop_step it saves the
    // per-step owner-state permutes and stack remapping and the separate leaf rounds through the FIFO
    // (C1: the trapped mirror paths' last bounces).  Called with the whole wave active.
    auto lone_walk = [&](const uint64_t own) {
        // 1, 2 or up to 4 owners (wave-uniform): the whole wave, its halves or its quarters work for
        // them, group g for the g-th lowest owner lane (with 3 owners the last quarter idles)
        const int nown = __popcll(own);
        const int hshift = nown == 1 ? 6 : (nown == 2 ? 5 : 4), hs = 1 << hshift;
        const int grp = (int)lane >> hshift;
        const int hb = grp << hshift;
        const int r = (int)lane - hb;  // worker rank
        const uint64_t gmask = hs == 64 ? ~0ull : (((1ull << hs) - 1) << hb);
        // this group's owner's ray, cull bounds and closest hit, by cross-lane permute (per-lane
        // copies: uniform copies of the owners' values would need ~40 SGPRs per owner, spilled)
        const uint64_t own1 = own & (own - 1), own2 = own1 & (own1 - 1), own3 = own2 & (own2 - 1);
        const uint64_t mine_o = grp == 0 ? own : (grp == 1 ? own1 : (grp == 2 ? own2 : own3));
        const bool has_owner = mine_o != 0;
        const int ow = has_owner ? (int)__builtin_ctzll(mine_o) : (int)lane;
        auto p64 = [&](double v) { return __shfl(v, ow); };
        auto p32 = [&](float v) { return __shfl(v, ow); };
        auto pi = [&](int v) { return __shfl(v, ow); };
        RayPre op;
        op.o = mk(p64(pre.o.x), p64(pre.o.y), p64(pre.o.z));
        op.d = mk(p64(pre.d.x), p64(pre.d.y), p64(pre.d.z));
        op.sx = p64(pre.sx);
        op.sy = p64(pre.sy);
        op.pdz = p64(pre.pdz);
        op.flags = pi(pre.flags);
        Ray32 ry;
        ry.ox = p32(pre32.ox); ry.oy = p32(pre32.oy); ry.oz = p32(pre32.oz);
        ry.ix = p32(pre32.ix); ry.iy = p32(pre32.iy); ry.iz = p32(pre32.iz);
        ry.nx = p32(pre32.nx); ry.ny = p32(pre32.ny); ry.nz = p32(pre32.nz);
        ry.e2 = p32(pre32.e2);
        float cf = p32(cull_far);
        const float cb = p32(cull_behind);
        const int cobj = pi(cur_object);
        int bkind = pi(best.kind), bindex = pi(best.index), bobject = pi(best.object);
        uint32_t brank = (uint32_t)pi((int)best.rank);
        double bd = p64(best.d);
        // frontier entry f of this half: row f / hs, column hb + f % hs of the wave's stack words
        auto fr = [&](int f) -> StackT& {
            return st_node[(f >> hshift) * 256 + (tid & ~63) + hb + (f & (hs - 1))];
        };
        const int cap = hs * STACK;
        // a batch pushes at most 3 net entries per entry taken and stays below `safe`; above it, one
        // entry per iteration is a depth-first walk of one subtree, which needs at most the per-lane
        // walk's stack (< STACK) plus one word per level (it pushes every hit child), < 2 * STACK
        const int safe = cap - 4 * STACK;
        int32_t* const leaves = &wl_tri[wbase + grp * (hs * kPend)];  // <= 1 per worker per step
        static_assert(kPend >= 1, "each group's share of the wave FIFO holds a step's leaves");
        // the owner's current node, permuted with the whole wave active: ds_bpermute reads 0 from a
        // source lane outside exec, so a permute inside `r == 0` (lanes 0 / 32 only) would start
        // the walk at node 0 whenever the owner is another lane
        const int start = pi(node);
        if (r == 0) fr(0) = (uint32_t)start;
        int n = has_owner ? 1 : 0;  // this group's frontier size
        while (true) {
            const bool act = n > 0;
            if (__ballot(act) == 0) break;
            if (!act) continue;
            VR_MARK("lone_step");
            VR_CPN(0, true);  // lone-walk iterations (per half)
            if (n > cap - 4) {  // cannot happen (above); a device error rather than a stray LDS write
                atomicOr(A.error_flag, 1);
                n = 0;
                continue;
            }
            // four workers per node, one child each: a quarter of the per-worker instructions of
            // one worker per node (C1 2.15 -> 1.60 ms, profiles/r05/lone/ab_split_c1.jsonl)
            const int tw = hs >> 2;
            int t = n < tw ? n : tw;
            if (n + 3 * t > safe) t = (safe - n) / 3 > 1 ? (safe - n) / 3 : 1;
            const int slot = r >> 2, k = r & 3;
            const int my = slot < t ? (int)fr(n - 1 - slot) : -1;
            n -= t;
            bool ih = false, lh = false;
            int c = 0;
            int32_t le = 0;
            if (my >= 0) {
                const Node4& nd = node_at(my);
                c = nd.child[k];
                float f, g;
                bool maybe, sure;
                slab32_flags(nd.box[k], ry, f, g, maybe, sure);
                const bool pass = c != kEmptyChild && maybe && !(f > cf || g < cb);
                ih = pass && c >= 0;
                lh = pass && c < 0;
                le = (~c) | ((pass && !sure) ? INT32_MIN : 0);
            }
            int nl = 0;  // hit leaves, in (node, child slot) order
            {
                const uint64_t mi = __ballot(ih) & gmask, ml = __ballot(lh) & gmask;
                if (ih) fr(n + (int)lanes_below(mi)) = (uint32_t)c;
                if (lh) leaves[(int)lanes_below(ml)] = le;
                n += (int)__popcll(mi);
                nl = (int)__popcll(ml);
            }
            for (int b = 0; b < nl; b += hs) {  // nl is uniform per half: the halves branch apart
                VR_MARK("lone_leaf");
                VR_CPN(1, true);  // lone-walk leaf rounds (per half)
                const bool mine = r < nl - b;
                double d = -1.0;
                uint64_t key = 0;
                if (mine) {
                    const int e = leaves[b + r];
                    const int tri = e & 0x7fffffff;
                    const TriVerts tv = load_tri(tri_at(tri));
                    double bb3[3];
                    d = triangle_distance(tv, op, bb3);
                    if (e < 0 && d >= 0.0) {  // the leaf's f32 box test was too close to call
                        double bb[6], lo, hi;
#pragma unroll
                        for (int a = 0; a < 3; ++a) {
                            bb[2 * a] = fmin(fmin(tv.v[a], tv.v[3 + a]), tv.v[6 + a]);
                            bb[2 * a + 1] = fmax(fmax(tv.v[a], tv.v[3 + a]), tv.v[6 + a]);
                        }
                        if (!slab(bb, op, lo, hi)) d = -1.0;
                    }
                    key = ((uint64_t)(uint32_t)tv.rank << 32) | (uint32_t)tri;
                }
                const bool hit = mine && d >= 0.0;
                const uint64_t hm = __ballot(hit) & gmask;
                if (hm == 0) continue;
                // the round's candidate over this half: the minimum distance (non-negative, so its
                // bits order as integers), and at it the highest rank (its triangle in the low half);
                // most rounds have one hit, taken by one permute
                const uint64_t db = hit ? (uint64_t)__double_as_longlong(d) : ~0ull;
                uint64_t dmin, kmax;
                if (__popcll(hm) == 1) {
                    const int src = (int)__builtin_ctzll(hm);
                    dmin = __shfl(db, src);
                    kmax = __shfl(key, src);
                } else {
                    dmin = db;
                    for (int sh = hs >> 1; sh >= 1; sh >>= 1) {
                        const uint64_t w = __shfl_xor(dmin, sh);
                        dmin = w < dmin ? w : dmin;
                    }
                    kmax = hit && db == dmin ? key : 0ull;
                    for (int sh = hs >> 1; sh >= 1; sh >>= 1) {
                        const uint64_t w = __shfl_xor(kmax, sh);
                        kmax = w > kmax ? w : kmax;
                    }
                }
                const double dd = __longlong_as_double((long long)dmin);
                const uint32_t rk = (uint32_t)(kmax >> 32);
                // takes_hit for the owner
                const bool closer = !bkind | (dd < bd);
                const bool tie = (dd == bd) & ((bobject == cobj) ? (rk > brank) : (cobj < bobject));
                if (closer | tie) {
                    bd = dd;
                    bkind = kTri;
                    bindex = (int)(uint32_t)kmax;
                    brank = rk;
                    bobject = cobj;
                    cf = round_away_f32(bd + S.margin * (1.0 + fabs(bd)) + margin_of(ry));  // set_cull_far
                }
            }
        }
        // each owner takes its group's results (from the group's first lane: the owners below it
        // count its group)
        const int src = (int)lanes_below(own) << hshift;
        const double rd = __shfl(bd, src);
        const int rkind = __shfl(bkind, src), rindex = __shfl(bindex, src), robject = __shfl(bobject, src);
        const uint32_t rrank = (uint32_t)__shfl((int)brank, src);
        const float rcf = __shfl(cf, src);
        if ((own >> lane) & 1ull) {
            best.d = rd;
            best.kind = rkind;
            best.index = rindex;
            best.rank = rrank;
            best.object = robject;
            cull_far = rcf;
            node = -1;
            sp = 0;
        }
    };
    while (true) {
        // ---------------------------------------------------------------- phase A: shade
        // repeated while some lane's new ray was resolved without BVH work (sky misses, rays
        // that only meet the plane or spheres), so those lanes do not idle through phase B
        VR_CP_PHASE_A();
        for (int rep = 0; rep < A.phase_a_reps; ++rep) {
            VR_MARK("phaseA_top");
            __builtin_amdgcn_s_setprio(kPrioA);
            if (COUNT && first_active_lane()) cnt.outer_slots += 64;
            VR_STAMP(5);
            // shading is deferred while fewer than shade_min lanes have a hit to shade and other
            // lanes still traverse: the deferred lanes wait (state kTraversed) and the next phase
            // A shades them with more lanes busy (misses are finished at once either way)
            bool shade_now = true, finish_now = true;
            if constexpr (TRACE) {
                if (state == kTraversed) {  // the ray's closest hit, then the next ray
                    double* h = A.probe_hits + 2 * (uint64_t)px;
                    __builtin_nontemporal_store(best.d, &h[0]);
                    __builtin_nontemporal_store(__longlong_as_double(
                        (long long)(((uint64_t)(uint32_t)best.object << 32) | ((uint32_t)best.index << 2) | (uint32_t)best.kind)), &h[1]);
                    ++s_idx;
                    state = kNeedRay;
                }
            } else if (A.shade_min | A.miss_min) {
                const bool idle = lanes_ieq(state, kTraversing) == 0;
                const uint64_t done_trav = lanes_ieq(state, kTraversed);
                const int nhit = __popcll(done_trav & lanes_ine((int)best.kind, (int)kNone));
                const int nmiss = __popcll(done_trav & lanes_ieq((int)best.kind, (int)kNone));
                shade_now = nhit >= (int)A.shade_min || idle;
                finish_now = nmiss >= (int)A.miss_min || idle;
            }
            if (!TRACE && state == kTraversed && (best.kind == kNone ? finish_now : shade_now)) {
                VR_MARK("traversed");
                // one call site for shade(): two inlined copies would both run whenever a wave
                // holds camera-ray hits and bounce hits at once
                bool go = false;
                fin = false;
#ifdef VR_DEBUG_PIX  // debug builds: one sample's traced rays and closest hits, for tools/debug_path.py
                if ((A.start_row + py) * A.width + (A.start_column + px) == (uint64_t)VR_DEBUG_PIX &&
                    A.first_sample + s_idx == (uint64_t)VR_DEBUG_SMP)
                    printf("vrdbg %d %d %d %llx %llx %llx %llx %llx %llx %llx %d\n", depth, (int)best.kind, best.index,
                           (unsigned long long)__double_as_longlong(best.d),
                           (unsigned long long)__double_as_longlong(pre.o.x), (unsigned long long)__double_as_longlong(pre.o.y),
                           (unsigned long long)__double_as_longlong(pre.o.z), (unsigned long long)__double_as_longlong(pre.d.x),
                           (unsigned long long)__double_as_longlong(pre.d.y), (unsigned long long)__double_as_longlong(pre.d.z),
                           best.kind == kTri ? (int)best.rank : -1);
#endif
                if (WHITTED && depth >= 0) {
                    if (!best.kind) {
                        finish(lambda, Acc);  // the continuation missed: photon.scale_intensity(0)
                    } else {
                        Acc = Acc + Wb;
                        T = Wa;
                        depth += 1;
                        go = true;
                    }
                } else if (depth < 0) {
                    if (!best.kind) {
                        finish(0.0, 0.0);  // camera ray missed: photon {0, 0} (camera.rs:110-113)
                    } else {
                        flags |= 1;
                        lambda = 380.0 + (740.0 - 380.0) * rng.standard();  // Photon::random_wavelength
                        T = 1.0; Acc = 0.0; T0 = 1.0; Acc0 = 0.0; b0 = 0.0;
                        depth = 0;
                        go = true;
                    }
                } else if (!best.kind) {
                    finish(lambda, Acc + T * sky_intensity(wo_y, lambda, &S.materials[S.sky_row]));  // simple_random_integrator.rs:43-46
                } else {
                    depth += 1;
                    if (depth == kRecursionLimit) {  // integrate(.., 0) returns {0, 0}: lambda becomes 0
                        flags |= 2;
                        // the innermost photon's intensity 0 times the lambda-0 throughput: + 0
                        // when finite, NaN when a level's pdf * |cos| was (the reference's 0 * NaN);
                        // DARK0 scenes are NaN-free (host), where every lambda-0 level is 0 * I + b
                        finish(0.0, DARK0 ? b0 : Acc0 + T0 * 0.0);
                    } else {
                        go = true;
                    }
                }
                if (go) shade();
                if (fin) store_photon(fin_wl, fin_I);
            }
            VR_STAMP(0);
            VR_MARK("refill_check");
            // refill: lanes whose item is exhausted take the next items (one atomic per wave)
            while (true) {
                const bool need = state == kNeedRay && s_idx >= s_end;
                const uint64_t m = lanes_ieq(state, kNeedRay) & lanes_uge(s_idx, s_end);
                if (m == 0) break;
                VR_SEC(7);
                VR_MARK("refill");
                const unsigned leader = (unsigned)__builtin_ctzll(m);
                const uint32_t rank = (uint32_t)lanes_below(m);
                unsigned long long base = 0;
                bool take = need;
                if (A.grab == 0) {
                    if (lane == leader) base = atomicAdd(A.queue, (unsigned long long)__popcll(m));
                    base = __shfl(base, (int)leader);
                } else {
                    // wave-private slice of the queue: one atomic per `grab` items
                    if (w_next >= w_end) {
                        if (lane == leader) base = atomicAdd(A.queue, (unsigned long long)A.grab);
                        w_next = uniform64(__shfl(base, (int)leader));
                        w_end = w_next + A.grab;
                    }
                    const uint64_t avail = w_end - w_next;
                    base = w_next;
                    take = need && rank < avail;
                    const uint64_t want = (uint64_t)__popcll(m);
                    w_next = uniform64(w_next + (want < avail ? want : avail));
                }
                if (TRACE && take) {  // a work item is one ray of probe_rays
                    const uint64_t g = base + rank;
                    if (g >= A.probe_n) {
                        state = kDone;
                    } else {
                        px = (uint32_t)g;
                        s_idx = 0;
                        s_end = 1;
                    }
                } else if (take) {
                    const uint64_t g = base + rank;
                    if (g >= items) {
                        state = kDone;
                    } else {
                        // g = (chunk_i * blocks + blk) * 64 + l; g >> 6 < 2^32 (the host caps
                        // a launch's items), quotients by f64 reciprocal, corrected by one
                        const uint32_t gb = (uint32_t)(g >> 6), l = (uint32_t)(g & 63);
                        uint32_t chunk_i;
                        int32_t rem;
                        if (A.item_order) {
                            // block-major: g = (blk * R + chunk_i) * 64 + l, R = the items per pixel
                            // -- the waves in flight work on few blocks at a time (see RenderArgs)
                            const uint32_t R = (uint32_t)(rounds + tail_of(A));
                            uint32_t bi = (uint32_t)((double)gb * rcp_R);
                            int32_t c = (int32_t)(gb - bi * R);
                            if (c < 0) { --bi; c += (int32_t)R; }
                            if (c >= (int32_t)R) { ++bi; c -= (int32_t)R; }
                            rem = (int32_t)bi;
                            chunk_i = (uint32_t)c;
                        } else {
                            const uint32_t nblk = (uint32_t)(per_chunk >> 6);
                            chunk_i = (uint32_t)((double)gb * rcp_live);
                            rem = (int32_t)(gb - chunk_i * nblk);
                            if (rem < 0) { --chunk_i; rem += (int32_t)nblk; }
                            if (rem >= (int32_t)nblk) { ++chunk_i; rem -= (int32_t)nblk; }
                        }
                        const uint32_t blk = A.live_blocks ? A.live_blocks[rem] : (uint32_t)rem;
                        uint32_t by = (uint32_t)((double)blk * A.rcp_bw);
                        int32_t bx = (int32_t)(blk - by * bw);
                        if (bx < 0) { --by; bx += (int32_t)bw; }
                        if (bx >= (int32_t)bw) { ++by; bx -= (int32_t)bw; }
                        const uint32_t x = (uint32_t)bx * 8 + (l & 7), y = by * 8 + (l >> 3);
                        // else padding: take another item (blocks whose camera rays all miss every
                        // object are not in the item space; their samples are the photon {0, 0},
                        // applied by the ordered reduce without staged data)
                        if (x < A.tile_width && y < A.tile_height) {
                            px = x;
                            py = y;
                            if (chunk_i < rounds) {
                                s_idx = chunk_i * A.chunk;
                                s_end = min(bulk, s_idx + A.chunk);
                            } else {
                                s_idx = bulk + (uint32_t)(chunk_i - rounds);
                                s_end = s_idx + 1;
                            }
                        }
                    }
                }
            }
            VR_STAMP(1);
            if (TRACE && state == kNeedRay) {
                const double* r = A.probe_rays + 6 * (uint64_t)px;
                pre.o = mk(__builtin_nontemporal_load(&r[0]), __builtin_nontemporal_load(&r[1]),
                           __builtin_nontemporal_load(&r[2]));
                pre.d = mk(__builtin_nontemporal_load(&r[3]), __builtin_nontemporal_load(&r[4]),
                           __builtin_nontemporal_load(&r[5]));
                state = kRayReady;
            } else if (state == kNeedRay) {
                const uint64_t row = A.start_row + py, col = A.start_column + px;
                rng.reset(stream_base_keyed(A.seed_key, row * A.width + col, A.first_sample + s_idx));
                // ImageSampler (camera.rs:24-66): film (w/h, 1) or (1, w/h); x's draw first
                VR_SEC(4);
                VR_MARK("camera");
                // film_w * (1 / w), film_w * 0.5, ... are per-launch constants (host: make_args)
                const double ux = rng.standard();
                const double uy = rng.standard();
                const double x = ((double)col + ux) * A.film[0] - A.film[1];
                const double y = ((double)(A.height - (row + 1)) + uy) * A.film[2] - A.film[3];
                depth = -1;
                bounces = 0;
                flags = 0;
                pre.o = mk(S.camera[0], S.camera[1], S.camera[2]);
                pre.d = normalize(mk(x, y, 1.0));
                state = kRayReady;
            }
            if (state == kRayReady) {
                VR_SEC(5);
                VR_MARK("begin_ray");
                begin_ray();
            }
            VR_STAMP(2);

            if (lanes_ieq(state, kTraversed) == 0) break;
        }
        if (lanes_ine(state, kDone) == 0) break;
        const bool tail = lanes_ieq(state, kDone) != 0;  // wave-uniform, fixed through phase B
        (void)tail;
        VR_CP(0);
        // ---------------------------------------------------------------- phase B: traverse
#if VR_WATCHDOG  // debug builds: a wave stuck in phase B prints its lanes' state and stops
        uint32_t wd = 0;
#endif
        do {
#if VR_WATCHDOG
            if (++wd > (1u << 20)) {
                printf("vr watchdog: block %u lane %u state %d node %d sp %d np %d q %u..%u bvh %d\n", blockIdx.x,
                       lane, (int)state, node, sp, (int)np, q_head, q_tail, bvh_i);
                atomicOr(A.error_flag, 1);
                state = kDone;
                break;
            }
#endif
            if (COUNT && first_active_lane()) cnt.trav_slots += 64;
            VR_STAMP(5);
            VR_MARK("phaseB_top");
            __builtin_amdgcn_s_setprio(kPrioNode);
            // node step (4-wide node), while the wave FIFO has room for four more leaves per lane
            bool lq[4] = {false, false, false, false};  // leaf children this lane queues in this step
            int32_t lent[4];
            bool coop = false;
            if constexpr (COOP) {
                if (A.coop && tail) {  // some lane of the wave is done: the queue is exhausted
                    const uint64_t live = __ballot(state != kDone);
                    const int nlive = __popcll(live);
                    // A.coop: owners served (1 or 2); to start, every live path must have bounced
                    // A.coop_bounces times.  Once on, it stays on for the wave: an owner's stack may
                    // span other lanes' columns, and the live set only shrinks (a live lane may still
                    // start a new path from the wave's slice, with its own empty stack)
                    if (!coop_on)
                        coop_on = nlive >= 1 && nlive <= (int)A.coop &&
                                  (__ballot(state != kDone && bounces >= (int)A.coop_bounces) == live);
                    coop = coop_on && nlive >= 1;
                    VR_CP(3);
                    VR_CP_TAIL(nlive);
                    if (coop) {
                        // the traversing paths' walks of their BVHs at once when nothing is pending
                        const uint64_t busy = lanes_ieq(state, kTraversing);
                        const uint64_t fresh = busy & lanes_ige(node, 0) & lanes_ieq(sp, 0) & lanes_ieq(np, 0);
                        if (A.lone_walk && busy != 0 && fresh == busy && __popcll(busy) <= 4 && q_head == q_tail) {
                            VR_CPN(3, true);
                            lone_walk(busy);
                        } else if (nlive <= 2) {
                            coop_step(live);
                        } else {
                            // 3 or 4 live paths with pending work: per-lane steps until every one of
                            // them is fresh again (each bounce's start), then their whole walks at once
                            coop = false;
                        }
                    }
                    VR_CP(1);
                }
            }
            if (COUNT) {  // how full this iteration's node step is (the headroom of merging waves)
                const int n = VR_ROOM ? __popcll(lanes_ieq(state, kTraversing) & lanes_ige(node, 0)) : 0;
                if (first_active_lane()) step_hist[n == 0 ? 0 : 1 + (n - 1) / 8]++;
            }
            // VR_NODE_STEPS (2) node steps per iteration: the second, with its leaf append, before the
            // leaf-round check, the next-BVH step and the loop condition, for the lanes still at a node
            // while the FIFO has room -- half the iterations' bookkeeping (round 6: C3 38.96 -> 38.13 ms,
            // C5 2048^2 @16 17.16 -> 16.34 ms, C2 -3.6 %; 3 steps: C3 38.24, C5 16.12 ms;
            // profiles/r06/steps/).  The order of node visits and leaf tests changes, the records do not
            // (every step and leaf round is order-independent)
            for (int nst = 0; nst < VR_NODE_STEPS; ++nst) {
                if (nst > 0) {
                    if (coop || (lanes_ieq(state, kTraversing) & lanes_ige(node, 0)) == 0 || !VR_ROOM) break;
#pragma unroll
                    for (int k = 0; k < 4; ++k) lq[k] = false;
                    if (COUNT && first_active_lane()) cnt.trav_slots += 64;
                }
                if (!coop && state == kTraversing && node >= 0 && VR_ROOM) {
                    VR_MARK("node_step");
                    // 32-bit byte offset from the scalar base (node < 2^25 unless BIG): the load's saddr form,
                    // no 64-bit address arithmetic per step
                    const Node4& nd = node_at(node);
                    if (COUNT) cnt.node_visits++;
                    int c[4];
                    float f[4];
                    // per-child bits: descend / queue (f32 hit or too close to call, not culled), and
                    // too close to call.  An interior child too close to call is descended: its box is
                    // a superset of its leaves' boxes, so walking it only costs work (DESIGN.md section
                    // 5); a leaf child too close to call is queued with bit 31 set and its exact f64 box
                    // test runs in the leaf round, beside the triangle test (the f32 bounds tlo / thi
                    // enclose the exact interval either way, so the f32 cull stays conservative)
                    uint32_t hm = 0, xm = 0;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        c[k] = nd.child[k];
                        float g;
                        bool maybe, sure;
                        slab32_flags(nd.box[k], pre32, f[k], g, maybe, sure);
                        const bool live = c[k] != kEmptyChild;
                        if (COUNT && live) cnt.box_tests++;
                        const bool pass = live && maybe && !(f[k] > cull_far || g < cull_behind);
                        hm |= pass ? 1u << k : 0u;
                        xm |= (pass && !sure) ? 1u << k : 0u;
                    }
                    // leaf children: their triangles go to the wave FIFO, appended after the step by all
                    // lanes at once
                    // interior children near-first: one 32-bit key per child, the entry distance's high
                    // bits (clamped below at 0: non-negative f32 bits order like the values) over the
                    // child's node index (A.sort_mask: the low bits, wide enough for every wide node), so
                    // the sorting network is integer min / max and the index rides along; 0xffffffff
                    // (or any key with bit 31 set) marks "not descended".  Only the visiting order depends on the key.
                    const uint32_t smask = A.sort_mask;
                    uint32_t key[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const bool h = (hm >> k) & 1u;
                        lent[k] = (~c[k]) | (((xm >> k) & 1u) ? INT32_MIN : 0);
                        lq[k] = h && c[k] < 0;
                        // a leaf or empty child's index is negative: its key has bit 31 set as it is
                        // (negative distances, -0 and negative NaNs clamp to 0 as integers; +inf and
                        // positive NaNs keep bit 31 clear: a hit child is never dropped)
                        uint32_t kb = ((uint32_t)max(__float_as_int(f[k]), 0) & ~smask) | (uint32_t)c[k];
                        asm volatile("" : "+v"(kb));  // computed for every lane: a select, not a branch
                        key[k] = h ? kb : 0xffffffffu;
                    }
                    auto cas = [&](int i, int j) {
                        const uint32_t ki = key[i], kj = key[j];
                        key[i] = ki < kj ? ki : kj;
                        key[j] = ki < kj ? kj : ki;
                    };
                    cas(0, 1);
                    cas(2, 3);
                    cas(0, 2);
                    cas(1, 3);
                    cas(1, 2);
                    if (key[0] < 0x80000000u) {
                        // farthest first, so the nearest remaining pops first (writes at sp are
                        // unconditional: the stack holds one spare entry)
                        // (sp advances by 1 + (key >> 31 arithmetic): 1 for a descended child, 0 else)
                        int32_t adv[4];
#pragma unroll
                        for (int k = 1; k < 4; ++k) {
                            adv[k] = (int32_t)key[k] >> 31;
                            asm volatile("" : "+v"(adv[k]));  // keeps the shift: LLVM would rebuild it as not + shift
                        }
                        st_node[sp * 256 + tid] = key[3] & smask;
                        sp += 1 + adv[3];
                        st_node[sp * 256 + tid] = key[2] & smask;
                        sp += 1 + adv[2];
                        st_node[sp * 256 + tid] = key[1] & smask;
                        sp += 1 + adv[1];
                        node = (int)(key[0] & smask);
                    } else if (sp > 0) {
                        --sp;
                        node = (int)st_node[sp * 256 + tid];
                    } else {
                        node = -1;  // this BVH is walked; its pending leaves remain
                    }
                }
                VR_STAMP(3);
                VR_MARK("leaf_check");
                __builtin_amdgcn_s_setprio(kPrioLeaf);
                // append this step's leaves to the wave FIFO in (child slot, lane) order (skipped when no
                // lane met a leaf: main -1.3 %, C5 -4.5 %)
                const uint64_t lqm[4] = {__ballot(lq[0]), __ballot(lq[1]), __ballot(lq[2]), __ballot(lq[3])};
                if ((lqm[0] | lqm[1] | lqm[2] | lqm[3]) != 0)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const bool lh = lq[k];
                    const uint64_t m = lqm[k];
                    if (lh) {
                        const uint32_t pos = (q_tail + (uint32_t)lanes_below(m)) & (kWaveList - 1);
                        wl_tri[wbase + pos] = lent[k];
                        wl_own[wbase + pos] = (uint8_t)lane;
                    }
                    q_tail += (uint32_t)__popcll(m);
                    np += lh ? 1 : 0;
                }
                q_tail = __builtin_amdgcn_readfirstlane(q_tail);
            }
            // leaf round: leaf_threshold (64) queued leaves -- every lane busy --, or enough lanes (or
            // all) are stalled on theirs
            const uint32_t queued = q_tail - q_head;
            if (queued != 0) {
                // the launch's tail (the queue is exhausted: some lane of the wave is done) with few
                // lanes still traversing (long paths alone in their wave): test their leaves at once,
                // so the hits found tighten the distance cull of the rest of the walk -- waiting for
                // a full round would walk the whole tree unculled
                const uint64_t trav = lanes_ieq(state, kTraversing);
                const bool room = VR_ROOM;  // wave-uniform
                const uint64_t at_node = trav & lanes_ige(node, 0);
                const uint64_t stalled_m = lanes_igt(np, 0) & (room ? ~lanes_ige(node, 0) : exec_mask());
                const bool few = coop || (tail && __popcll(trav) <= (int)A.leaf_few);
                if (queued >= A.leaf_threshold || few || __popcll(stalled_m) >= (int)A.leaf_stall ||
                    !room || at_node == 0) {
                    VR_SEC(0);
                    VR_MARK("leaf_test");
                    VR_CP(3);
                    VR_CPN(1, coop_on);
                    leaf_round(queued < 64u ? queued : 64u);
                    q_head = __builtin_amdgcn_readfirstlane(q_head + (queued < 64u ? queued : 64u));
                    VR_CP(2);
                }
            }
            VR_STAMP(4);
            if (state == kTraversing && node < 0 && np == 0) {
                VR_SEC(8);
                VR_MARK("next_bvh");
                ++bvh_i;
                if (!start_bvhs()) state = kTraversed;
            }
            VR_CP(3);
        } while (lanes_ieq(state, kTraversing) != 0 &&
                 __popcll(lanes_ieq(state, kTraversed)) < (int)A.shade_threshold);
    }
    VR_CP_DUMP();
#undef VR_CP
#undef VR_CPN
#undef VR_CP_PHASE_A
#undef VR_CP_TAIL
#undef VR_CP_DUMP

    if (COUNT) {
        atomicAdd(&A.counters[kCntBoxTests], (unsigned long long)cnt.box_tests);
        atomicAdd(&A.counters[kCntNodeVisits], (unsigned long long)cnt.node_visits);
        atomicAdd(&A.counters[kCntTriangleTests], (unsigned long long)cnt.tri_tests);
        atomicAdd(&A.counters[kCntRays], (unsigned long long)cnt.rays);
        atomicAdd(&A.counters[kCntShadedTriangles], (unsigned long long)cnt.shaded);
        atomicAdd(&A.counters[kCntSamples], (unsigned long long)samples_done);
        atomicAdd(&A.counters[kCntTraversalSlots], (unsigned long long)cnt.trav_slots);
        atomicAdd(&A.counters[kCntOuterSlots], (unsigned long long)cnt.outer_slots);
        atomicAdd(&A.counters[kCntExactBoxes], (unsigned long long)cnt.exact_boxes);
        VR_STAMP(5);
        if (first_active_lane())
            for (int i = 0; i < 6; ++i) atomicAdd(&A.counters[kCntCycles + i], (unsigned long long)cyc[i]);
        for (int i = 0; i < 3; ++i)
            if (prim_cnt[i]) atomicAdd(&A.counters[kCntPrimTests + i], (unsigned long long)prim_cnt[i]);
        for (int i = 0; i < 9; ++i) {  // each lane counted the executions it led
            if (sec[i]) atomicAdd(&A.counters[kCntSections + i], (unsigned long long)sec[i]);
            if (step_hist[i]) atomicAdd(&A.counters[kCntStepHist + i], (unsigned long long)step_hist[i]);
        }
        if (A.wg_times) {
            __syncthreads();
            if (tid == 0) A.wg_times[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

#undef VR_STAMP
#undef VR_SEC

// Camera-frustum test of the tile's 8x8 pixel blocks (one thread per block).  The camera rays of a
// block start at the camera and pass through the film rectangle its pixels' sample squares cover
// (camera.rs:24-66: x = (col + u) fw/w - fw/2, y = (h - row - 1 + v) fh/h - fh/2, u, v in [0, 1),
// direction (x, y, 1) normalised).  A block is culled only when every such line provably misses
// every object, with margins far beyond the f64 rounding of the reference's tests:
//  * a plane (plane.rs:49-75): its t = num / dn is negative for every ray -- num and n . (x, y, 1)
//    of opposite signs at all four corners of the rectangle (a linear function: its extremes),
//    each by more than 1e-9 of its magnitude scale;
//  * a BVH root box (a ray that misses the box misses every triangle in it) wholly in front of the
//    camera: the bounding rectangle of its corners' film projections (x/z, y/z), widened by 1e-6,
//    misses the block's film rectangle;
//  * a sphere, or a root box through its bounding sphere: the camera is outside it and the angle
//    between the sphere's centre and the axis of the block's cone of directions exceeds the cone's
//    half-angle (attained at a corner) plus the sphere's angular radius plus 1e-6 rad.
// Each sample of a culled block is then exactly the missed camera ray's photon {0, 0}, whatever
// its random draws.
__device__ __forceinline__ double vr_angle(V3 a, V3 b) {
    return atan2(sqrt(dot(cross(a, b), cross(a, b))), dot(a, b));
}
__global__ __launch_bounds__(256) void block_cull_kernel(RenderArgs A, const Prim* prims, const Bvh* bvhs,
                                                         uint8_t* mask) {
    const uint32_t bw = (uint32_t)((A.tile_width + 7) / 8), bh = (uint32_t)((A.tile_height + 7) / 8);
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b >= bw * bh) return;
    const uint32_t bx = b % bw, by = b / bw;
    const double c0 = (double)(A.start_column + 8 * (uint64_t)bx);
    const double c1 = (double)(A.start_column + min((uint64_t)8 * bx + 8, A.tile_width));
    const double r0 = (double)(A.start_row + 8 * (uint64_t)by);
    const double r1 = (double)(A.start_row + min((uint64_t)8 * by + 8, A.tile_height));
    const double H = (double)A.height;
    const double xa = c0 * A.film[0] - A.film[1], xb = c1 * A.film[0] - A.film[1];
    const double ya = (H - r1) * A.film[2] - A.film[3], yb = (H - r0) * A.film[2] - A.film[3];
    const double mx = 1e-9 * (fabs(xa) + fabs(xb) + 1.0), my = 1e-9 * (fabs(ya) + fabs(yb) + 1.0);
    const double xlo = fmin(xa, xb) - mx, xhi = fmax(xa, xb) + mx;
    const double ylo = fmin(ya, yb) - my, yhi = fmax(ya, yb) + my;
    const V3 pc[4] = {mk(xlo, ylo, 1.0), mk(xhi, ylo, 1.0), mk(xlo, yhi, 1.0), mk(xhi, yhi, 1.0)};
    V3 axis = mk(0.0, 0.0, 0.0);
    for (int i = 0; i < 4; ++i) axis = add(axis, normalize(pc[i]));
    axis = normalize(axis);
    double half = 0.0;
    for (int i = 0; i < 4; ++i) half = fmax(half, vr_angle(axis, pc[i]));
    const V3 o = mk(A.scene.camera[0], A.scene.camera[1], A.scene.camera[2]);
    // a sphere (centre c, radius r) every ray of the block misses
    auto sphere_clear = [&](V3 c, double r) {
        const V3 v = sub(c, o);
        const double dist = sqrt(dot(v, v));
        if (!(dist > r * (1.0 + 1e-6) + 1e-9)) return false;
        return vr_angle(axis, v) > half + asin(fmin(1.0, r / dist)) + 1e-6;
    };
    bool clear = true;
    for (int i = 0; i < A.scene.prim_count && clear; ++i) {
        const Prim& pr = prims[i];
        const V3 c = ldv(pr.vec);
        if (pr.kind == 0) {
            const V3 q = ldv(pr.pre);
            const double num = dot(sub(q, o), c);
            const double nn = sqrt(dot(c, c));
            const double tol = 1e-9 * nn * (sqrt(dot(q, q)) + sqrt(dot(o, o)) + 1.0);
            if (!(fabs(num) > tol)) {
                clear = false;
                break;
            }
            for (int k = 0; k < 4; ++k) {
                const double dn = dot(pc[k], c);
                const double t = 1e-9 * nn * sqrt(dot(pc[k], pc[k]));
                if (!(num > 0.0 ? dn < -t : dn > t)) clear = false;
            }
        } else {
            clear = sphere_clear(c, pr.scalar);
        }
    }
    for (int i = 0; i < A.scene.bvh_count && clear; ++i) {
        const Bvh& bv = bvhs[i];
        if (bv.root4 == INT32_MIN) continue;  // an empty mesh never hits
        const double* bb = bv.root_box;
        // a box wholly in front of the camera: the directions that reach it project (x/z, y/z)
        // into the bounding rectangle of its corners' projections; clear when that rectangle,
        // widened by 1e-6 of its scale, misses the block's film rectangle
        double ulo = INFINITY, uhi = -INFINITY, vlo = INFINITY, vhi = -INFINITY;
        bool front = true;
        for (int k = 0; k < 8; ++k) {
            const double px = bb[k & 1] - o.x, py = bb[2 + ((k >> 1) & 1)] - o.y, pz = bb[4 + (k >> 2)] - o.z;
            front = front && pz > 1e-6 * (fabs(px) + fabs(py) + fabs(pz));
            ulo = fmin(ulo, px / pz);
            uhi = fmax(uhi, px / pz);
            vlo = fmin(vlo, py / pz);
            vhi = fmax(vhi, py / pz);
        }
        if (front) {
            const double mu = 1e-6 * (fabs(ulo) + fabs(uhi) + 1.0), mv = 1e-6 * (fabs(vlo) + fabs(vhi) + 1.0);
            if (uhi + mu < xlo || ulo - mu > xhi || vhi + mv < ylo || vlo - mv > yhi) continue;
        }
        const V3 c = mk(0.5 * (bb[0] + bb[1]), 0.5 * (bb[2] + bb[3]), 0.5 * (bb[4] + bb[5]));
        const V3 e = mk(bb[1] - bb[0], bb[3] - bb[2], bb[5] - bb[4]);
        clear = sphere_clear(c, 0.5 * sqrt(dot(e, e)) * (1.0 + 1e-9) + 1e-12);
    }
    mask[b] = clear ? 1 : 0;
}

// The live blocks of a cull mask (one workgroup: each thread counts a contiguous run of the index
// space, an LDS scan gives the runs' offsets, then each thread writes its run's live blocks).  The
// index space is the blocks in row-major order, or (morton) the Z-order curve over the tile's
// blocks padded to a power-of-two square: with block-major work items (RenderArgs::item_order) the
// waves in flight then cover a compact square of the image instead of a strip.
__device__ __forceinline__ uint32_t vr_compact1by1(uint32_t x) {
    x &= 0x55555555u;
    x = (x | (x >> 1)) & 0x33333333u;
    x = (x | (x >> 2)) & 0x0F0F0F0Fu;
    x = (x | (x >> 4)) & 0x00FF00FFu;
    x = (x | (x >> 8)) & 0x0000FFFFu;
    return x;
}
__global__ __launch_bounds__(1024) void block_compact_kernel(const uint8_t* mask, uint32_t bw, uint32_t bh,
                                                              uint32_t side, uint32_t* live, uint32_t* count) {
    __shared__ uint32_t part[1024];
    const uint32_t n = side ? side * side : bw * bh;  // the index space
    auto block_of = [&](uint32_t i) -> int64_t {    // the live block at index i, or -1
        uint32_t b = i;
        if (side) {
            const uint32_t x = vr_compact1by1(i), y = vr_compact1by1(i >> 1);
            if (x >= bw || y >= bh) return -1;
            b = y * bw + x;
        }
        return mask[b] == 0 ? (int64_t)b : -1;
    };
    const uint32_t tid = threadIdx.x, per = (n + 1023) / 1024;
    const uint32_t lo = min(n, tid * per), hi = min(n, lo + per);
    uint32_t c = 0;
    for (uint32_t i = lo; i < hi; ++i) c += block_of(i) >= 0;
    part[tid] = c;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {  // inclusive Hillis-Steele scan
        const uint32_t v = tid >= d ? part[tid - d] : 0u;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    uint32_t off = part[tid] - c;
    for (uint32_t i = lo; i < hi; ++i) {
        const int64_t b = block_of(i);
        if (b >= 0) live[off++] = (uint32_t)b;
    }
    if (tid == 1023) *count = part[1023];
}

#ifndef VR_REDUCE_BATCH  // samples whose colours the ordered reduce computes together
#define VR_REDUCE_BATCH 4
#endif
typedef double d2 __attribute__((ext_vector_type(2)));
// accumulation_buffer.rs:44-60 (update_pixel with weight 1.0), one thread per pixel, samples in
// order: the same Kahan sequence the reference applies call by call.
__constant__ double c_exp_tab[64] = VR_EXP_TABLE_INIT;
__global__ __launch_bounds__(256) void accumulate_kernel(double* state, const double* staging, uint64_t npix,
                                                         uint32_t spp, uint32_t accumulate, const uint8_t* mask,
                                                         uint64_t tile_width, const uint32_t* stage_tag,
                                                         uint32_t stage_gen, int32_t* error_flag) {
    // Debug builds (-DVR_STAGE_GUARD): every staged photon the reduce reads must carry this pass's
    // generation -- a slot the render kernel did not write in this pass is a device error (error
    // word bit 3, VR_ERROR_DEVICE "staging guard").  The invariant it checks: the reduce reads
    // slot (s, p) exactly for the pixels p < npix outside culled blocks and the samples s < spp,
    // and the render kernel's item space covers exactly those (pixel, sample) pairs.
#ifdef VR_STAGE_GUARD
    auto guard = [&](uint32_t s, uint64_t p) {
        if (stage_tag[(uint64_t)s * npix + p] != stage_gen) {
            if (atomicOr(error_flag, 8) == 0)
                printf("vr staging guard: pixel %llu sample %u tag %u, pass generation %u\n", (unsigned long long)p, s,
                       stage_tag[(uint64_t)s * npix + p], stage_gen);
            atomicOr(error_flag, 8);
        }
    };
#define VR_GUARD(s, p) guard(s, p)
#else
#define VR_GUARD(s, p) ((void)stage_tag, (void)stage_gen, (void)error_flag)
#endif
    __shared__ double etab[64];  // 2^(j/64) for the lobes' exp (vr_exp_table.h)
    if (threadIdx.x < 64) etab[threadIdx.x] = c_exp_tab[threadIdx.x];
    __syncthreads();
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= npix) return;
    // records (vr_layout.h): the pixel's sums {X, Y, Z, weight} at state[4p], its Kahan
    // compensations at state[4 npix + 4p] -- 32 B each, one dwordx4 pair per half
    d2* const rs = reinterpret_cast<d2*>(state + 4 * p);
    d2* const rb = reinterpret_cast<d2*>(state + 4 * npix + 4 * p);
    double sum[3] = {0.0, 0.0, 0.0}, bias[3] = {0.0, 0.0, 0.0}, w = 0.0, wb = 0.0;
    if (accumulate) {
        const d2 s0 = rs[0], s1 = rs[1], b0 = rb[0], b1 = rb[1];
        sum[0] = s0.x; sum[1] = s0.y; sum[2] = s1.x; w = s1.y;
        bias[0] = b0.x; bias[1] = b0.y; bias[2] = b1.x; wb = b1.y;
    }
    // update_pixel for one sample (the Kahan chain is sequential in s)
    auto update = [&](const double c[3]) {
        const double wy = 1.0 - wb;
        const double wt = w + wy;
        wb = (wt - w) - wy;
        w = wt;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double y = c[k] * 1.0 - bias[k];
            const double t = sum[k] + y;
            bias[k] = (t - sum[k]) - y;
            sum[k] = t;
        }
    };
    // the colours of kB samples are independent (7 exp() each): computed together, then folded in
    // order -- the same operations as one at a time, with kB-fold instruction-level parallelism
    constexpr uint32_t kB = VR_REDUCE_BATCH;
    uint32_t s = 0;
    if (mask) {
        const uint64_t py = p / tile_width, px = p - py * tile_width;
        if (mask[(py >> 3) * ((tile_width + 7) >> 3) + (px >> 3)]) {
            // a culled block (block_cull_kernel): every sample is the photon {0, 0}, colour +0.
            // From a fresh record the Kahan chain has a closed form: colour y = +0 * 1 - +0 = +0
            // keeps sums and compensations +0, and the weight counts 1, 2, .., spp exactly with
            // compensation (n + 1 - n) - 1 = 0 (spp < 2^32 < 2^53)
            if (!accumulate) {
                w = (double)spp;
                s = spp;
            }
            const double z[3] = {0.0, 0.0, 0.0};
            for (; s < spp; ++s) update(z);
        }
    }
    for (; s + kB <= spp; s += kB) {
        double c[kB][3];
        d2 v[kB];
        uint64_t bits = 0;  // OR of the batch's photon bits: 0 iff all four are {+0, +0}
#pragma unroll
        for (uint32_t j = 0; j < kB; ++j) {
            // final photon {wavelength, intensity}: one 16-B non-temporal load
            VR_GUARD(s + j, p);
            v[j] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(staging) + ((uint64_t)(s + j) * npix + p));
            bits |= (uint64_t)__double_as_longlong(v[j].x) | (uint64_t)__double_as_longlong(v[j].y);
        }
        // the lanes with some nonzero photon bit, as one 64-bit compare into a lane mask.  (Not a
        // compare of a zero-extended bool "dark" with 0: hipcc of ROCm 7.2 folded that into the
        // mask of the dark lanes -- the opposite polarity -- once this loop was split in two, so a
        // wave with ANY dark lane zeroed every lane's colours; DESIGN.md section 8, "the staging
        // invariant")
        if (__builtin_amdgcn_uicmpl(bits, 0ull, 33 /* ne */) == 0) {
            // a missed camera ray's photon {+0, +0} (camera.rs:110-113): every lobe is positive at
            // 0 nm, so its colour is (+0, +0, +0) exactly -- the wave skips the 28 exp when all
            // its photons are such (rows of pixels that see no geometry)
#pragma unroll
            for (uint32_t j = 0; j < kB; ++j) c[j][0] = c[j][1] = c[j][2] = 0.0;
        } else {
#pragma unroll
            for (uint32_t j = 0; j < kB; ++j) {
                const double wl = v[j].x, I = v[j].y;
                const double Is = I * 360.0;                     // photon.rs:26-28, camera.rs:121-126
                const V3 cx = xyz_for_wavelength_tab(wl, etab);  // colour_xyz.rs:31-35
                c[j][0] = cx.x * Is;
                c[j][1] = cx.y * Is;
                c[j][2] = cx.z * Is;
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < kB; ++j) update(c[j]);
    }
    for (; s < spp; ++s) {
        VR_GUARD(s, p);
        const d2 v = __builtin_nontemporal_load(reinterpret_cast<const d2*>(staging) + ((uint64_t)s * npix + p));
        const double wl = v.x, I = v.y;
        const double Is = I * 360.0;
        const V3 cx = xyz_for_wavelength_tab(wl, etab);
        const double c[3] = {cx.x * Is, cx.y * Is, cx.z * Is};
        update(c);
    }
    rs[0] = d2{sum[0], sum[1]};
    rs[1] = d2{sum[2], w};
    rb[0] = d2{bias[0], bias[1]};
    rb[1] = d2{bias[2], wb};
}
#undef VR_GUARD

template <int STACK>
__global__ __launch_bounds__(256) void trace_kernel(TraceArgs A) {
    __shared__ int st_node[STACK * 256];
    __shared__ float st_t[STACK * 256];
    const int tid = threadIdx.x;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + tid;
    if (i >= A.n) return;
    Ray r;
    r.o = ldv(A.origins + 3 * i);
    r.d = ldv(A.directions + 3 * i);
    RayPre pre = prepare(r);
    Counts cnt = {0, 0, 0, 0, 0, 0, 0, 0};
    Best best = closest_hit<STACK, false>(A.scene, pre, st_node, st_t, tid, cnt);
    vr_hit_record* out = (vr_hit_record*)A.out + i;
    out->valid = best.kind != kNone;
    if (!best.kind) return;
    HitInfo h;
    hit_info(A.scene, best, pre, h);
    out->object = best.object;
    out->primitive = best.kind == kPrim ? A.scene.prims[best.index].position : best.index;
    if (best.kind == kTri) {
        for (int b = 0; b < A.scene.bvh_count; ++b)
            if (A.scene.bvhs[b].object == best.object)
                out->primitive = A.scene.tris[best.index].rank - A.scene.bvhs[b].tri_base;  // reference leaf position
    }
    out->distance = best.d;
    out->location[0] = h.loc.x; out->location[1] = h.loc.y; out->location[2] = h.loc.z;
    out->normal[0] = h.normal.x; out->normal[1] = h.normal.y; out->normal[2] = h.normal.z;
    out->tangent[0] = h.tangent.x; out->tangent[1] = h.tangent.y; out->tangent[2] = h.tangent.z;
    out->cotangent[0] = h.cotangent.x; out->cotangent[1] = h.cotangent.y; out->cotangent[2] = h.cotangent.z;
    out->retro[0] = h.retro.x; out->retro[1] = h.retro.y; out->retro[2] = h.retro.z;
}

}  // namespace dev

// ----------------------------------------------------------------------------------------------
// Host-side launch wrappers
// ----------------------------------------------------------------------------------------------
static hipError_t launch_reduce(const RenderArgs& a, hipStream_t s, hipEvent_t mid) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (mid) {  // between the render kernel and the ordered reduce (timed launches)
        e = hipEventRecord(mid, s);
        if (e != hipSuccess) return e;
    }
    const uint64_t npix = a.tile_width * a.tile_height;
    hipLaunchKernelGGL(dev::accumulate_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, s, a.state,
                       (const double*)a.staging, npix, a.spp, a.accumulate, a.block_mask, a.tile_width,
                       a.stage_tag, a.stage_gen, a.error_flag);
    return hipGetLastError();
}

template <int STACK>
static hipError_t launch_render_t(const RenderArgs& a, const LaunchChoice& c, int grid_limit, hipStream_t s,
                                  hipEvent_t mid) {
    // persistent waves: enough workgroups to fill the chip, each wave loops over work items
    const uint64_t items = dev::render_items(a, ((a.tile_width + 7) / 8) * ((a.tile_height + 7) / 8) * 64);
    const uint64_t want = (items + 255) / 256;
    dim3 grid((unsigned)(want < (uint64_t)grid_limit ? want : (uint64_t)grid_limit)), block(256);
    const bool recording = c.recording, counting = c.counting;
#define VR_K(...) hipLaunchKernelGGL((dev::render_kernel<__VA_ARGS__>), grid, block, 0, s, a, a.scene.prims, \
                                     a.scene.materials, a.scene.bvhs)
    if (c.big) {
        // 64-bit load offsets (scenes past 4 GB of triangles or 2^25 wide nodes): the general
        // kernels only (DARK0 = false and every material kind are always correct, only slower), in
        // the deepest stack class only (launch_render)
        if constexpr (STACK != 48) return hipErrorInvalidValue;
        else if (a.scene.integrator == 1) {
            if (recording) VR_K(STACK, false, true, false, 3, 3, true, false, true);
            else if (counting) VR_K(STACK, true, false, false, 3, 3, true, false, true);
            else VR_K(STACK, false, false, false, 3, 3, true, false, true);
        } else {
            if (recording) VR_K(STACK, false, true, false, 3, 3, false, false, true);
            else if (counting) VR_K(STACK, true, false, false, 3, 3, false, false, true);
            else VR_K(STACK, false, false, false, 3, 3, false, false, true);
        }
        return launch_reduce(a, s, mid);
    }
    if (a.scene.integrator == 1) {  // WhittedIntegrator: the general-material kernel
        if (recording) VR_K(STACK, false, true, true, 3, 3, true);
        else if (counting) VR_K(STACK, true, false, true, 3, 3, true);
        else VR_K(STACK, false, false, true, 3, 3, true);
        return launch_reduce(a, s, mid);
    }
    // kinds present (bit 0 Lambertian, 1 reflective, 2 Phong or dielectric) -> specialisation:
    // Lambertian-only (1), reflective-only (2) or the general kernel (3)
    int mats = (c.mats == 1 || c.mats == 2) ? c.mats : 3;
    if (!c.dark0) mats = 3;  // the general kernel
#ifdef VR_TUNING_VARIANTS  // experiment hooks of tuning builds only (tools/variants.py)
    // 1..4 = force that many waves per SIMD (default 3); 5 / 6: 16-bit LDS stack entries (trees below
    // 65,536 wide nodes only) at 4 / 3 waves per SIMD; VR_FORCE_MATS: the material specialisation
    const char* ve = getenv("VR_KERNEL_VARIANT");
    const int variant = ve ? atoi(ve) : 0;
    if (const char* fm = getenv("VR_FORCE_MATS")) mats = atoi(fm);
#define VR_MODES(D, M)                                          \
    if (recording) VR_K(STACK, false, true, D, M, 3);           \
    else if (counting) VR_K(STACK, true, false, D, M, 3);       \
    else if (variant == 1) VR_K(STACK, false, false, D, M, 1);  \
    else if (variant == 2) VR_K(STACK, false, false, D, M, 2);  \
    else if (variant == 4) VR_K(STACK, false, false, D, M, 4);  \
    else if (variant == 5 && STACK == 32) VR_K(STACK, false, false, D, M, 4, false, false, false, false, true); \
    else if (variant == 6 && STACK == 32) VR_K(STACK, false, false, D, M, 3, false, false, false, false, true); \
    else if (s16) VR_K(STACK_S16, false, false, D, M, 3, false, false, false, false, true); \
    else VR_K(STACK, false, false, D, M, 3)
#else
#define VR_MODES(D, M)                                                                  \
    if (recording) VR_K(STACK, false, true, D, M, 3);                                   \
    else if (counting) VR_K(STACK, true, false, D, M, 3);                               \
    else if (s16) VR_K(STACK_S16, false, false, D, M, 3, false, false, false, false, true); \
    else VR_K(STACK, false, false, D, M, 3)
#endif
    // the cooperative-tail instantiations: launches the host marks (RenderArgs::coop: small launches
    // of scenes with a reflective material)
#ifndef VR_COOP_MINW  // their waves per SIMD (2: no spills; C1 -9 %)
#define VR_COOP_MINW 2
#endif
    const bool coop = c.coop;
    // 16-bit LDS stack entries (LaunchChoice::s16: trees below 65,536 wide nodes) for the timed
    // kernels of the 24 / 32 stack classes: half the stack's LDS at the same 3 waves per SIMD, C3
    // 39.22 -> 38.71 ms, 1024^2 @64 10.83 -> 10.58 ms, records bit-identical (profiles/r06/occ)
    constexpr int STACK_S16 = STACK <= 32 ? STACK : 32;  // (never launched for the 48 class)
    const bool s16 = c.s16 && STACK <= 32;
    if (!c.dark0) {
        VR_MODES(false, 3);
    } else if (mats == 1) {
        VR_MODES(true, 1);
    } else if (mats == 2) {
        if (coop) VR_K(STACK, false, false, true, 2, VR_COOP_MINW, false, true);
        else VR_MODES(true, 2);
    } else {
        if (coop) VR_K(STACK, false, false, true, 3, VR_COOP_MINW, false, true);
        else VR_MODES(true, 3);
    }
#undef VR_MODES
#undef VR_K
    return launch_reduce(a, s, mid);
}

int launch_block_cull(const RenderArgs& a, uint8_t* mask, void* stream) {
    const uint64_t blocks = ((a.tile_width + 7) / 8) * ((a.tile_height + 7) / 8);
    if (blocks == 0) return 0;
    hipLaunchKernelGGL(dev::block_cull_kernel, dim3((unsigned)((blocks + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       a, a.scene.prims, a.scene.bvhs, mask);
    return (int)hipGetLastError();
}

int launch_block_compact(const uint8_t* mask, uint32_t bw, uint32_t bh, bool morton, uint32_t* live, uint32_t* count,
                         void* stream) {
    // Z-order only for near-square block grids (the padded square at most 4x the blocks)
    uint32_t side = 0;
    if (morton) {
        side = 1;
        while (side < bw || side < bh) side <<= 1;
        if ((uint64_t)side * side > 4ull * bw * bh || side > 32768) side = 0;
    }
    hipLaunchKernelGGL(dev::block_compact_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, mask, bw, bh, side, live,
                       count);
    return (int)hipGetLastError();
}

int launch_render(const RenderArgs& a, const LaunchChoice& c, int grid_limit, void* stream, void* mid_event) {
    hipStream_t s = (hipStream_t)stream;
    hipEvent_t mid = (hipEvent_t)mid_event;
    if (a.tile_width == 0 || a.tile_height == 0 || a.spp == 0) return 0;
    hipError_t e;
    // the 64-bit-offset kernels exist in the deepest stack class only (a scene that needs them is
    // far larger than any whose tree fits the smaller classes; more LDS is only fewer waves)
    if (c.big && c.stack_depth <= 48) e = launch_render_t<48>(a, c, grid_limit, s, mid);
    else if (c.stack_depth <= 24) e = launch_render_t<24>(a, c, grid_limit, s, mid);
    else if (c.stack_depth <= 32) e = launch_render_t<32>(a, c, grid_limit, s, mid);
    else if (c.stack_depth <= 48) e = launch_render_t<48>(a, c, grid_limit, s, mid);
    else return -1000;
    return (int)e;
}

int launch_trace(const TraceArgs& a, int stack_depth, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (a.n == 0) return 0;
    dim3 grid((unsigned)((a.n + 255) / 256)), block(256);
    if (stack_depth <= 24) hipLaunchKernelGGL(dev::trace_kernel<24>, grid, block, 0, s, a);
    else if (stack_depth <= 32) hipLaunchKernelGGL(dev::trace_kernel<32>, grid, block, 0, s, a);
    else if (stack_depth <= 48) hipLaunchKernelGGL(dev::trace_kernel<48>, grid, block, 0, s, a);
    else return -1000;
    return (int)hipGetLastError();
}

#ifdef VR_SPLIT_PROBE
// analysis builds: the traversal-only instantiations (TRACE) of the render kernel over a ray buffer,
// at `minw` waves per SIMD, with 32- or 16-bit LDS stack entries
int launch_trace_probe(const RenderArgs& a, int stack_depth, int minw, bool s16, int grid, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    dim3 g((unsigned)grid), b(256);
#define VR_KT(ST, MW, S16_)                                                                                    \
    hipLaunchKernelGGL((dev::render_kernel<ST, false, false, true, 3, MW, false, false, false, true, S16_>), g, b, \
                       0, s, a, a.scene.prims, a.scene.materials, a.scene.bvhs)
    if (stack_depth > 32) return -1000;
    if (s16) {
        if (minw == 3) VR_KT(32, 3, true);
        else if (minw == 4) VR_KT(32, 4, true);
        else if (minw == 5) VR_KT(32, 5, true);
        else if (minw == 6) VR_KT(32, 6, true);
        else return -1001;
    } else {
        if (minw == 3) VR_KT(32, 3, false);
        else if (minw == 4) VR_KT(32, 4, false);
        else return -1001;
    }
#undef VR_KT
    return (int)hipGetLastError();
}
#endif

const char* device_error_string(int code) {
    if (code == -1000) return "BVH deeper than the largest traversal stack (48)";
    return hipGetErrorString((hipError_t)code);
}

}  // namespace vr

// vr_build.hip -- BoundingVolumeHierarchy::build_from_slice (bounding_volume_hierarchy.rs:38-74)
// on the device, producing exactly the host build's flattened BVH (vr_host.cpp BvhBuilder):
// the same pre-order node array, the same leaf order, the same child boxes.
//
// The reference splits every node of n > 1 triangles at n / 2 after sorting its triangles by
// box centre along the largest extent of the node's bounds (util/axis_aligned_bounding_box.rs:
// 76-99).  The tree's SHAPE therefore depends on n alone: a node over [lo, hi) has children
// [lo, lo + n/2) and [lo + n/2, hi), its left child is node me + 1 and its right child node
// me + n/2 in pre-order.  Only the split axes and the permutation depend on the geometry, so
// the build runs level by level over the whole mesh:
//
//   1. bounds of every segment of the level (rocprim segmented reduce of triangle boxes,
//      NaN-ignoring min/max like f64::min/max) -> the parent's child box and link, the axis;
//   2. one key per position: (segment start, centre[axis] as an order-preserving u64, input
//      index) -- positions already in leaves keep their own start as the segment;
//   3. rocprim merge sort of the keys = every segment sorted by (centre, input index) at once
//      (the host build breaks centre ties by input index too; pdqsort's order of equal keys is
//      unspecified in the reference);
//   4. the permutation follows the sorted keys.
//
// Work per level is O(n log n) device work; for the 1M-triangle C5 mesh the build replaces a
// host std::sort recursion.  Scenes whose vertices contain NaN use the host build (the
// reference's comparator maps NaN to Equal, which is not a strict order to reproduce).
#include <hip/hip_runtime.h>

#include <rocprim/device/device_merge_sort.hpp>
#include <rocprim/device/device_segmented_reduce.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include <math.h>
#include <stdint.h>

#include <vector>

#include "vr_layout.h"

namespace vr {
namespace build {

struct BoxD {
    double mn[3], mx[3];
};
struct BoxUnion {  // Interval::union (interval.rs:66-77): f64::min / f64::max ignore NaN
    __host__ __device__ BoxD operator()(const BoxD& a, const BoxD& b) const {
        BoxD r;
        for (int i = 0; i < 3; ++i) {
            r.mn[i] = fmin(a.mn[i], b.mn[i]);
            r.mx[i] = fmax(a.mx[i], b.mx[i]);
        }
        return r;
    }
};
struct SortKey {
    uint64_t k;     // centre[axis], order-preserving bits (-0 folded into +0: they compare equal)
    uint32_t seg;   // start position of the segment (orders segments, keeps fixed leaves in place)
    uint32_t orig;  // input triangle index: the tie-break
};
struct KeyLess {
    __host__ __device__ bool operator()(const SortKey& a, const SortKey& b) const {
        if (a.seg != b.seg) return a.seg < b.seg;
        if (a.k != b.k) return a.k < b.k;
        return a.orig < b.orig;
    }
};
struct BoxOfPosition {  // position -> box of the triangle currently there
    const BoxD* boxes;
    const uint32_t* perm;
    __host__ __device__ BoxD operator()(uint32_t pos) const { return boxes[perm[pos]]; }
};

__device__ __forceinline__ uint64_t order_bits(double x) {
    if (x == 0.0) x = 0.0;
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// BoundingBox::from_points over the 3 vertices (triangle.rs:101-105) and centre() (:79-84)
__global__ void prim_boxes_kernel(const double* verts, uint32_t n, BoxD* boxes, double* centres, uint32_t* perm) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    BoxD b;
    for (int c = 0; c < 3; ++c) b.mn[c] = b.mx[c] = verts[9 * (uint64_t)t + c];
    for (int k = 1; k < 3; ++k)
        for (int c = 0; c < 3; ++c) {
            const double v = verts[9 * (uint64_t)t + 3 * k + c];
            b.mn[c] = fmin(b.mn[c], v);
            b.mx[c] = fmax(b.mx[c], v);
        }
    boxes[t] = b;
    for (int c = 0; c < 3; ++c) centres[3 * (uint64_t)t + c] = (b.mn[c] + b.mx[c]) / 2.0;
    perm[t] = t;
}

// largest_dimension (util/axis_aligned_bounding_box.rs:76-99): size -1 for a flat axis, ties keep
// the earlier axis
__device__ __forceinline__ int largest_dimension(const BoxD& b) {
    int acc = 0;
    double acc_size = 0.0;
    for (int i = 0; i < 3; ++i) {
        const double size = b.mn[i] == b.mx[i] ? -1.0 : b.mx[i] - b.mn[i];
        if (size > acc_size) {
            acc = i;
            acc_size = size;
        }
    }
    return acc;
}

struct LevelSeg {
    uint32_t lo, hi;
    int32_t node;    // pre-order interior index within the mesh (>= 0) or -1 (a leaf)
    int32_t parent;  // parent's interior index or -1 (the root)
    int32_t which;   // 0 left, 1 right child of the parent
    int32_t pad;
};

// child boxes and links into the parent; the split axis of interior segments
__global__ void write_level_kernel(const LevelSeg* segs, uint32_t nseg, const BoxD* bounds, Node* nodes,
                                   int32_t node_base, int32_t tri_base, int32_t* axis, double* root_box) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg) return;
    const LevelSeg g = segs[s];
    const BoxD b = bounds[s];
    double box[6];
    for (int i = 0; i < 3; ++i) {
        box[2 * i] = b.mn[i];
        box[2 * i + 1] = b.mx[i];
    }
    if (g.parent >= 0) {
        Node& p = nodes[g.parent];
        for (int i = 0; i < 6; ++i) p.box[g.which][i] = box[i];
        p.child[g.which] = g.node >= 0 ? node_base + g.node : ~(tri_base + (int32_t)g.lo);
    } else {
        for (int i = 0; i < 6; ++i) root_box[i] = box[i];
    }
    axis[s] = g.node >= 0 ? largest_dimension(b) : 0;
}

__global__ void keys_kernel(const LevelSeg* segs, uint32_t nseg, const int32_t* axis, const double* centres,
                            const uint32_t* perm, uint32_t n, SortKey* keys) {
    const uint32_t pos = blockIdx.x * blockDim.x + threadIdx.x;
    if (pos >= n) return;
    // the level's segments are disjoint and sorted by lo: the last one starting at or before pos
    uint32_t a = 0, b = nseg;
    while (b - a > 1) {
        const uint32_t m = (a + b) / 2;
        if (segs[m].lo <= pos) a = m;
        else b = m;
    }
    const LevelSeg g = segs[a];
    const uint32_t t = perm[pos];
    SortKey k;
    k.orig = t;
    if (g.lo <= pos && pos < g.hi && g.node >= 0) {
        k.seg = g.lo;
        k.k = order_bits(centres[3 * (uint64_t)t + axis[a]]);
    } else {  // a leaf (this level's or an earlier one's): stays where it is
        k.seg = pos;
        k.k = 0;
    }
    keys[pos] = k;
}

__global__ void scatter_kernel(const SortKey* keys, uint32_t n, uint32_t* perm) {
    const uint32_t pos = blockIdx.x * blockDim.x + threadIdx.x;
    if (pos < n) perm[pos] = keys[pos].orig;
}

// triangles and normals in leaf order
__global__ void gather_kernel(const double* verts, const double* norms, const uint32_t* perm, uint32_t n,
                              int32_t tri_base, TriVerts* tris, TriNormals* normals) {
    const uint32_t pos = blockIdx.x * blockDim.x + threadIdx.x;
    if (pos >= n) return;
    const uint64_t t = perm[pos];
    TriVerts tv;
    TriNormals tn;
    for (int i = 0; i < 9; ++i) {
        tv.v[i] = verts[9 * t + i];
        tn.n[i] = norms[9 * t + i];
    }
    tv.rank = tri_base + (int64_t)pos;  // this build IS the reference topology
    tn.pad = 0.0;
    tris[pos] = tv;
    normals[pos] = tn;
}

// The render kernel's 4-wide tree over a device-built binary tree: one thread per wide node
// gathers its child boxes from the binary nodes named by the host-made descriptor (desc[8i + k]:
// binary node * 2 + child for slot k, or -1; desc[8i + 4 + k]: the slot's child link) and writes
// them rounded outward to f32 (min toward -inf, max toward +inf: the host build's nextafter rule).
__global__ void fill_wide_kernel(const Node* bin, const int32_t* desc, uint64_t n4, Node4* out4) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    Node4 w;
    for (int k = 0; k < 4; ++k) {
        const int32_t src = desc[8 * i + k];
        w.child[k] = desc[8 * i + 4 + k];
        w.pad[k] = 0;
        for (int j = 0; j < 6; ++j) {
            const double v = src >= 0 ? bin[src >> 1].box[src & 1][j] : NAN;
            w.box[k][j] = src < 0 ? NAN : ((j & 1) ? __double2float_ru(v) : __double2float_rd(v));
        }
    }
    out4[i] = w;
}

// ------------------------------------------------------------------------------------------------
// The default traversal tree on the device (VR_SCENE_DEVICE_SAH): the binned-SAH binary tree of
// vr_host.cpp SahBuilder, built top-down one level at a time, one workgroup per segment of the
// level.  Its input is the reference-order triangle array the median build above leaves (each
// TriVerts carries its reference in-order rank, which breaks distance ties);
// its output is the SAH binary tree and the triangles permuted into its leaf order.  The tree
// differs from the host's only where the host's unstable std::partition / nth_element order equal
// keys: renders are bit-identical for any tree, only the work differs.
//
// Per segment [lo, hi) of positions (pos -> reference index perm[pos]):
//   1. the node box (union of the triangles' boxes) and the centroid bounds, reduced over the
//      workgroup; the box goes into the parent's child slot (or the root box);
//   2. 32 bins per axis over the centroid bounds: counts and bin boxes in LDS (64-bit atomics on
//      order-preserving bits of the doubles);
//   3. the split with the least area(left) * n_left + area(right) * n_right (axes and bins in
//      order, the first minimum wins -- the host's loops); none, or the depth cap of the
//      traversal stack reached (level + ceil(log2 n) >= 44, as the host): split at the middle;
//   4. a stable partition of the segment's positions into perm_out, then the two child segments
//      (node indices from an atomic counter; any numbering serves, the 4-wide collapse renumbers).
// ------------------------------------------------------------------------------------------------
struct SahSeg {
    uint32_t lo, hi;
    int32_t node;    // interior index (n >= 2) or -1
    int32_t parent;  // parent's interior index, -1 for the root
    int32_t which;   // child slot in the parent
    int32_t level;
};

constexpr int kSahBins = 32;

__device__ __forceinline__ uint64_t omin_bits(double x) { return order_bits(x); }
__device__ __forceinline__ double from_order_bits(uint64_t b) {
    const uint64_t r = (b >> 63) ? (b & 0x7FFFFFFFFFFFFFFFull) : ~b;
    return __longlong_as_double((long long)r);
}

// reference-order triangles -> per-position box and centroid (BoundingBox::from_points, centre())
__global__ void sah_prims_kernel(const TriVerts* tris, uint32_t n, BoxD* boxes, double* centres, uint32_t* perm) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const TriVerts tv = tris[t];
    BoxD b;
    for (int c = 0; c < 3; ++c) b.mn[c] = b.mx[c] = tv.v[c];
    for (int k = 1; k < 3; ++k)
        for (int c = 0; c < 3; ++c) {
            b.mn[c] = fmin(b.mn[c], tv.v[3 * k + c]);
            b.mx[c] = fmax(b.mx[c], tv.v[3 * k + c]);
        }
    boxes[t] = b;
    for (int c = 0; c < 3; ++c) centres[3 * (uint64_t)t + c] = (b.mn[c] + b.mx[c]) / 2.0;
    perm[t] = t;
}

__device__ __forceinline__ double sah_area(const double mn[3], const double mx[3]) {
    const double dx = mx[0] - mn[0], dy = mx[1] - mn[1], dz = mx[2] - mn[2];
    if (!(dx >= 0.0) || !(dy >= 0.0) || !(dz >= 0.0)) return 0.0;
    return 2.0 * (dx * dy + dy * dz + dz * dx);
}

__global__ __launch_bounds__(256) void sah_level_kernel(const SahSeg* segs, uint32_t nseg, const BoxD* boxes,
                                                        const double* centres, const uint32_t* perm_in,
                                                        uint32_t* perm_out, uint32_t* leaf_perm, Node* nodes,
                                                        int32_t node_base,
                                                        int32_t tri_base, double* root_box, SahSeg* next,
                                                        uint32_t* next_count, uint32_t* node_count,
                                                        uint32_t* max_level) {
    __shared__ double r_mn[4][6], r_mx[4][6];  // per wave: box min / max (0..2), centroid (3..5)
    __shared__ uint32_t cnt[3][kSahBins];
    __shared__ unsigned long long bmn[3][kSahBins][3], bmx[3][kSahBins][3];
    __shared__ int s_axis, s_bin;
    __shared__ double s_cmin[3], s_scale[3];
    __shared__ uint32_t s_nl, s_base_l, s_base_r, s_wave_l[4];
    const uint32_t si = blockIdx.x;
    if (si >= nseg) return;
    const SahSeg g = segs[si];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t n = g.hi - g.lo;
    // 1. node box and centroid bounds
    double mn[6], mx[6];
    for (int c = 0; c < 6; ++c) {
        mn[c] = INFINITY;
        mx[c] = -INFINITY;
    }
    for (uint32_t p = g.lo + tid; p < g.hi; p += 256) {
        const uint32_t r = perm_in[p];
        const BoxD b = boxes[r];
        for (int c = 0; c < 3; ++c) {
            mn[c] = fmin(mn[c], b.mn[c]);
            mx[c] = fmax(mx[c], b.mx[c]);
            const double ce = centres[3 * (uint64_t)r + c];
            mn[3 + c] = fmin(mn[3 + c], ce);
            mx[3 + c] = fmax(mx[3 + c], ce);
        }
    }
    for (int off = 32; off > 0; off >>= 1)
        for (int c = 0; c < 6; ++c) {
            mn[c] = fmin(mn[c], __shfl_xor(mn[c], off));
            mx[c] = fmax(mx[c], __shfl_xor(mx[c], off));
        }
    if (lane == 0)
        for (int c = 0; c < 6; ++c) {
            r_mn[wv][c] = mn[c];
            r_mx[wv][c] = mx[c];
        }
    for (uint32_t i = tid; i < 3 * kSahBins; i += 256) {
        cnt[i / kSahBins][i % kSahBins] = 0;
        for (int c = 0; c < 3; ++c) {
            bmn[i / kSahBins][i % kSahBins][c] = ~0ull;
            bmx[i / kSahBins][i % kSahBins][c] = 0ull;
        }
    }
    __syncthreads();
    for (int c = 0; c < 6; ++c) {
        mn[c] = fmin(fmin(r_mn[0][c], r_mn[1][c]), fmin(r_mn[2][c], r_mn[3][c]));
        mx[c] = fmax(fmax(r_mx[0][c], r_mx[1][c]), fmax(r_mx[2][c], r_mx[3][c]));
    }
    if (tid == 0) {
        double box[6];
        for (int c = 0; c < 3; ++c) {
            box[2 * c] = mn[c];
            box[2 * c + 1] = mx[c];
        }
        if (g.parent >= 0) {
            Node& pn = nodes[g.parent];
            for (int i = 0; i < 6; ++i) pn.box[g.which][i] = box[i];
            pn.child[g.which] = n >= 2 ? node_base + g.node : ~(tri_base + (int32_t)g.lo);
        } else {
            for (int i = 0; i < 6; ++i) root_box[i] = box[i];
        }
        atomicMax(max_level, (uint32_t)g.level + 1);
    }
    if (n < 2) {  // a leaf: its triangle's final position is lo
        if (tid == 0) leaf_perm[g.lo] = perm_in[g.lo];
        return;
    }
    // 2. binning (axes with a positive centroid extent)
    const int need = 32 - __clz((int)(n - 1));  // ceil(log2 n)
    const bool sah = g.level + need < 44;
    if (tid < 3) {
        const double ext = mx[3 + tid] - mn[3 + tid];
        s_cmin[tid] = mn[3 + tid];
        s_scale[tid] = ext > 0.0 ? kSahBins / ext : 0.0;
    }
    __syncthreads();
    if (sah) {
        for (uint32_t p = g.lo + tid; p < g.hi; p += 256) {
            const uint32_t r = perm_in[p];
            const BoxD b = boxes[r];
            for (int a = 0; a < 3; ++a) {
                if (!(s_scale[a] > 0.0)) continue;
                int k = (int)((centres[3 * (uint64_t)r + a] - s_cmin[a]) * s_scale[a]);
                k = k < 0 ? 0 : (k > kSahBins - 1 ? kSahBins - 1 : k);
                atomicAdd(&cnt[a][k], 1u);
                for (int c = 0; c < 3; ++c) {
                    atomicMin(&bmn[a][k][c], (unsigned long long)omin_bits(b.mn[c]));
                    atomicMax(&bmx[a][k][c], (unsigned long long)omin_bits(b.mx[c]));
                }
            }
        }
    }
    __syncthreads();
    // 3. the cheapest split (thread 0: 3 axes x 31 candidate planes)
    if (tid == 0) {
        int best_axis = -1, best_bin = -1;
        double best_cost = INFINITY;
        uint32_t best_nl = 0;
        for (int a = 0; sah && a < 3; ++a) {
            if (!(s_scale[a] > 0.0)) continue;
            double rarea[kSahBins];
            uint32_t rcnt[kSahBins];
            double amn[3] = {INFINITY, INFINITY, INFINITY}, amx[3] = {-INFINITY, -INFINITY, -INFINITY};
            uint32_t c = 0;
            for (int k = kSahBins - 1; k > 0; --k) {
                if (cnt[a][k])
                    for (int j = 0; j < 3; ++j) {
                        amn[j] = fmin(amn[j], from_order_bits(bmn[a][k][j]));
                        amx[j] = fmax(amx[j], from_order_bits(bmx[a][k][j]));
                    }
                c += cnt[a][k];
                rarea[k] = sah_area(amn, amx);
                rcnt[k] = c;
            }
            for (int j = 0; j < 3; ++j) {
                amn[j] = INFINITY;
                amx[j] = -INFINITY;
            }
            c = 0;
            for (int k = 0; k < kSahBins - 1; ++k) {
                if (cnt[a][k])
                    for (int j = 0; j < 3; ++j) {
                        amn[j] = fmin(amn[j], from_order_bits(bmn[a][k][j]));
                        amx[j] = fmax(amx[j], from_order_bits(bmx[a][k][j]));
                    }
                c += cnt[a][k];
                if (c == 0 || rcnt[k + 1] == 0) continue;
                const double cost = sah_area(amn, amx) * (double)c + rarea[k + 1] * (double)rcnt[k + 1];
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = a;
                    best_bin = k;
                    best_nl = c;
                }
            }
        }
        s_axis = best_axis;
        s_bin = best_bin;
        s_nl = best_axis >= 0 ? best_nl : n / 2;  // no split found / depth cap: the middle
        s_base_l = 0;
        s_base_r = 0;
    }
    __syncthreads();
    // 4. stable partition, 256 positions at a time
    const int axis = s_axis, bin = s_bin;
    const uint32_t nl = s_nl;
    for (uint32_t t0 = g.lo; t0 < g.hi; t0 += 256) {
        const uint32_t p = t0 + tid;
        const bool in = p < g.hi;
        uint32_t r = 0;
        bool left = false;
        if (in) {
            r = perm_in[p];
            if (axis >= 0) {
                int k = (int)((centres[3 * (uint64_t)r + axis] - s_cmin[axis]) * s_scale[axis]);
                k = k < 0 ? 0 : (k > kSahBins - 1 ? kSahBins - 1 : k);
                left = k <= bin;
            } else {
                left = p - g.lo < nl;
            }
        }
        const uint64_t ml = __ballot(in && left), mr = __ballot(in && !left);
        if (lane == 0) s_wave_l[wv] = (uint32_t)__popcll(ml) | ((uint32_t)__popcll(mr) << 16);
        __syncthreads();
        uint32_t bl = s_base_l, br = s_base_r;
        for (uint32_t w = 0; w < wv; ++w) {
            bl += s_wave_l[w] & 0xffff;
            br += s_wave_l[w] >> 16;
        }
        const uint64_t below = (1ull << lane) - 1;
        if (in) {
            if (left) perm_out[g.lo + bl + (uint32_t)__popcll(ml & below)] = r;
            else perm_out[g.lo + nl + br + (uint32_t)__popcll(mr & below)] = r;
        }
        __syncthreads();
        if (tid == 0) {
            for (int w = 0; w < 4; ++w) {
                s_base_l += s_wave_l[w] & 0xffff;
                s_base_r += s_wave_l[w] >> 16;
            }
        }
        __syncthreads();
    }
    // the child segments of the next level
    if (tid == 0) {
        const uint32_t nr = n - nl;
        const uint32_t slot = atomicAdd(next_count, 2u);
        const int32_t ln = nl >= 2 ? (int32_t)atomicAdd(node_count, 1u) : -1;
        const int32_t rn = nr >= 2 ? (int32_t)atomicAdd(node_count, 1u) : -1;
        next[slot] = {g.lo, g.lo + nl, ln, g.node, 0, g.level + 1};
        next[slot + 1] = {g.lo + nl, g.hi, rn, g.node, 1, g.level + 1};
    }
}

// the triangles and normals into the tree's leaf order (ranks ride along in TriVerts)
__global__ void sah_gather_kernel(const TriVerts* tin, const TriNormals* nin, const uint32_t* perm, uint32_t n,
                                  TriVerts* tout, TriNormals* nout) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    tout[p] = tin[perm[p]];
    nout[p] = nin[perm[p]];
}

}  // namespace build

#define VRB(call)                                 \
    do {                                          \
        hipError_t e_ = (call);                   \
        if (e_ != hipSuccess) return (int)e_;     \
    } while (0)

namespace {
struct DevBuf {
    void* p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    hipError_t alloc(size_t n) { return hipMalloc(&p, n ? n : 1); }
};
}  // namespace

// Builds one mesh's BVH into the scene's device arrays.  verts / norms: host [n][3][3] f64.
// nodes: the mesh's n - 1 interior nodes (pre-order, node_base-relative links made global);
// tris / normals: its n triangles in leaf order; leaf_order (host): input index per leaf;
// root_box (host, 6 f64); levels (host): tree depth.  Returns a hipError_t (0 = success).
int device_build_bvh(const double* verts, const double* norms, uint32_t n, int32_t node_base, int32_t tri_base,
                     Node* nodes, TriVerts* tris, TriNormals* normals, uint64_t* leaf_order, double* root_box,
                     int* levels, void* stream) {
    using namespace build;
    hipStream_t st = (hipStream_t)stream;
    // the tree's shape (depends on n only), level by level in pre-order
    std::vector<std::vector<LevelSeg>> lv;
    {
        std::vector<LevelSeg> cur = {{0, n, n > 1 ? 0 : -1, -1, 0, 0}};
        while (!cur.empty()) {
            std::vector<LevelSeg> next;
            for (const LevelSeg& g : cur) {
                if (g.node < 0) continue;
                const uint32_t size = g.hi - g.lo, half = size / 2, mid = g.lo + half;
                next.push_back({g.lo, mid, half > 1 ? g.node + 1 : -1, g.node, 0, 0});
                next.push_back({mid, g.hi, size - half > 1 ? g.node + (int32_t)half : -1, g.node, 1, 0});
            }
            lv.push_back(std::move(cur));
            cur = std::move(next);
        }
    }
    *levels = (int)lv.size();
    size_t max_seg = 1;
    for (auto& l : lv) max_seg = std::max(max_seg, l.size());

    DevBuf d_verts, d_norms, d_boxes, d_centres, d_perm, d_keys, d_keys2, d_segs, d_lo, d_hi, d_bounds, d_axis,
        d_root, d_temp;
    VRB(d_verts.alloc(sizeof(double) * 9 * (size_t)n));
    VRB(d_norms.alloc(sizeof(double) * 9 * (size_t)n));
    VRB(d_boxes.alloc(sizeof(BoxD) * (size_t)n));
    VRB(d_centres.alloc(sizeof(double) * 3 * (size_t)n));
    VRB(d_perm.alloc(sizeof(uint32_t) * (size_t)n));
    VRB(d_keys.alloc(sizeof(SortKey) * (size_t)n));
    VRB(d_keys2.alloc(sizeof(SortKey) * (size_t)n));
    VRB(d_segs.alloc(sizeof(LevelSeg) * max_seg));
    VRB(d_lo.alloc(sizeof(uint32_t) * max_seg));
    VRB(d_hi.alloc(sizeof(uint32_t) * max_seg));
    VRB(d_bounds.alloc(sizeof(BoxD) * max_seg));
    VRB(d_axis.alloc(sizeof(int32_t) * max_seg));
    VRB(d_root.alloc(sizeof(double) * 6));
    VRB(hipMemcpyAsync(d_verts.p, verts, sizeof(double) * 9 * (size_t)n, hipMemcpyHostToDevice, st));
    VRB(hipMemcpyAsync(d_norms.p, norms, sizeof(double) * 9 * (size_t)n, hipMemcpyHostToDevice, st));
    const dim3 blk(256);
    auto grid = [](uint64_t m) { return dim3((unsigned)((m + 255) / 256)); };
    BoxD* boxes = (BoxD*)d_boxes.p;
    uint32_t* perm = (uint32_t*)d_perm.p;
    SortKey* keys = (SortKey*)d_keys.p;
    SortKey* keys2 = (SortKey*)d_keys2.p;
    hipLaunchKernelGGL(prim_boxes_kernel, grid(n), blk, 0, st, (const double*)d_verts.p, n, boxes,
                       (double*)d_centres.p, perm);
    VRB(hipGetLastError());

    // temporary storage: the largest of the two primitives' needs
    auto box_in = rocprim::make_transform_iterator(rocprim::make_counting_iterator<uint32_t>(0),
                                                   BoxOfPosition{boxes, perm});
    BoxD empty;
    for (int i = 0; i < 3; ++i) {
        empty.mn[i] = INFINITY;
        empty.mx[i] = -INFINITY;
    }
    size_t t_red = 0, t_sort = 0;
    VRB(rocprim::segmented_reduce(nullptr, t_red, box_in, (BoxD*)d_bounds.p, (unsigned)max_seg, (uint32_t*)d_lo.p,
                                  (uint32_t*)d_hi.p, BoxUnion{}, empty, st));
    VRB(rocprim::merge_sort(nullptr, t_sort, keys, keys2, (size_t)n, KeyLess{}, st));
    VRB(d_temp.alloc(std::max(t_red, t_sort)));

    std::vector<uint32_t> lo, hi;
    for (size_t L = 0; L < lv.size(); ++L) {
        const std::vector<LevelSeg>& segs = lv[L];
        const uint32_t ns = (uint32_t)segs.size();
        lo.resize(ns);
        hi.resize(ns);
        bool interior = false;
        for (uint32_t i = 0; i < ns; ++i) {
            lo[i] = segs[i].lo;
            hi[i] = segs[i].hi;
            interior = interior || segs[i].node >= 0;
        }
        VRB(hipMemcpyAsync(d_segs.p, segs.data(), sizeof(LevelSeg) * ns, hipMemcpyHostToDevice, st));
        VRB(hipMemcpyAsync(d_lo.p, lo.data(), sizeof(uint32_t) * ns, hipMemcpyHostToDevice, st));
        VRB(hipMemcpyAsync(d_hi.p, hi.data(), sizeof(uint32_t) * ns, hipMemcpyHostToDevice, st));
        size_t tb = t_red;
        VRB(rocprim::segmented_reduce(d_temp.p, tb, box_in, (BoxD*)d_bounds.p, ns, (uint32_t*)d_lo.p,
                                      (uint32_t*)d_hi.p, BoxUnion{}, empty, st));
        hipLaunchKernelGGL(write_level_kernel, grid(ns), blk, 0, st, (const LevelSeg*)d_segs.p, ns,
                           (const BoxD*)d_bounds.p, nodes, node_base, tri_base, (int32_t*)d_axis.p,
                           (double*)d_root.p);
        VRB(hipGetLastError());
        if (!interior) continue;
        hipLaunchKernelGGL(keys_kernel, grid(n), blk, 0, st, (const LevelSeg*)d_segs.p, ns,
                           (const int32_t*)d_axis.p, (const double*)d_centres.p, (const uint32_t*)perm, n, keys);
        VRB(hipGetLastError());
        tb = t_sort;
        VRB(rocprim::merge_sort(d_temp.p, tb, keys, keys2, (size_t)n, KeyLess{}, st));
        hipLaunchKernelGGL(scatter_kernel, grid(n), blk, 0, st, (const SortKey*)keys2, n, perm);
        VRB(hipGetLastError());
    }
    hipLaunchKernelGGL(gather_kernel, grid(n), blk, 0, st, (const double*)d_verts.p, (const double*)d_norms.p,
                       (const uint32_t*)perm, n, tri_base, tris, normals);
    VRB(hipGetLastError());
    std::vector<uint32_t> p(n);
    VRB(hipMemcpyAsync(p.data(), perm, sizeof(uint32_t) * (size_t)n, hipMemcpyDeviceToHost, st));
    VRB(hipMemcpyAsync(root_box, d_root.p, sizeof(double) * 6, hipMemcpyDeviceToHost, st));
    VRB(hipStreamSynchronize(st));
    for (uint32_t i = 0; i < n; ++i) leaf_order[i] = p[i];
    return 0;
}

// The SAH traversal tree of one mesh whose triangles (tris / normals, n of them, reference leaf
// order with ranks) are already on the device: nodes[0 .. n-1) receive the binary tree (root at
// 0, links node_base-relative made global), tris / normals are permuted into its leaf order.
// root_box (host, 6 f64) and levels (host: depth) are returned.  Returns a hipError_t.
int device_build_sah(TriVerts* tris, TriNormals* normals, uint32_t n, int32_t node_base, int32_t tri_base,
                     Node* nodes, double* root_box, int* levels, void* stream) {
    using namespace build;
    hipStream_t st = (hipStream_t)stream;
    if (n < 2) return 0;
    DevBuf d_boxes, d_centres, d_perm, d_perm2, d_leaf, d_seg, d_seg2, d_ctr, d_root, d_tris, d_norms;
    VRB(d_boxes.alloc(sizeof(BoxD) * (size_t)n));
    VRB(d_centres.alloc(sizeof(double) * 3 * (size_t)n));
    VRB(d_perm.alloc(sizeof(uint32_t) * (size_t)n));
    VRB(d_perm2.alloc(sizeof(uint32_t) * (size_t)n));
    VRB(d_leaf.alloc(sizeof(uint32_t) * (size_t)n));
    VRB(hipMemsetAsync(nodes, 0, sizeof(Node) * (size_t)(n - 1), st));
    VRB(d_seg.alloc(sizeof(SahSeg) * (size_t)n));
    VRB(d_seg2.alloc(sizeof(SahSeg) * (size_t)n));
    VRB(d_ctr.alloc(sizeof(uint32_t) * 4));  // next segment count, node count, max level
    VRB(d_root.alloc(sizeof(double) * 6));
    const dim3 blk(256);
    auto grid = [](uint64_t m) { return dim3((unsigned)((m + 255) / 256)); };
    hipLaunchKernelGGL(sah_prims_kernel, grid(n), blk, 0, st, (const TriVerts*)tris, n, (BoxD*)d_boxes.p,
                       (double*)d_centres.p, (uint32_t*)d_perm.p);
    VRB(hipGetLastError());
    const SahSeg root = {0, n, 0, -1, 0, 0};
    VRB(hipMemcpyAsync(d_seg.p, &root, sizeof root, hipMemcpyHostToDevice, st));
    const uint32_t ctr0[4] = {0, 1, 0, 0};  // the root holds interior index 0
    VRB(hipMemcpyAsync(d_ctr.p, ctr0, sizeof ctr0, hipMemcpyHostToDevice, st));
    uint32_t* ctr = (uint32_t*)d_ctr.p;
    SahSeg *cur = (SahSeg*)d_seg.p, *nxt = (SahSeg*)d_seg2.p;
    uint32_t *pin = (uint32_t*)d_perm.p, *pout = (uint32_t*)d_perm2.p;
    uint32_t nseg = 1;
    while (nseg) {
        VRB(hipMemsetAsync(ctr, 0, sizeof(uint32_t), st));
        hipLaunchKernelGGL(sah_level_kernel, dim3(nseg), blk, 0, st, (const SahSeg*)cur, nseg,
                           (const BoxD*)d_boxes.p, (const double*)d_centres.p, (const uint32_t*)pin, pout,
                           (uint32_t*)d_leaf.p, nodes, node_base, tri_base, (double*)d_root.p, nxt, ctr, ctr + 1,
                           ctr + 2);
        VRB(hipGetLastError());
        VRB(hipMemcpyAsync(&nseg, ctr, sizeof nseg, hipMemcpyDeviceToHost, st));
        VRB(hipStreamSynchronize(st));
        std::swap(cur, nxt);
        std::swap(pin, pout);  // every position of an interior segment was partitioned into pout
    }
    uint32_t c[4];
    VRB(hipMemcpyAsync(c, ctr, sizeof c, hipMemcpyDeviceToHost, st));
    VRB(hipMemcpyAsync(root_box, d_root.p, sizeof(double) * 6, hipMemcpyDeviceToHost, st));
    // triangles into leaf order (through copies: the gather reads the reference order)
    VRB(d_tris.alloc(sizeof(TriVerts) * (size_t)n));
    VRB(d_norms.alloc(sizeof(TriNormals) * (size_t)n));
    VRB(hipMemcpyAsync(d_tris.p, tris, sizeof(TriVerts) * (size_t)n, hipMemcpyDeviceToDevice, st));
    VRB(hipMemcpyAsync(d_norms.p, normals, sizeof(TriNormals) * (size_t)n, hipMemcpyDeviceToDevice, st));
    hipLaunchKernelGGL(sah_gather_kernel, grid(n), blk, 0, st, (const TriVerts*)d_tris.p,
                       (const TriNormals*)d_norms.p, (const uint32_t*)d_leaf.p, n, tris, normals);
    VRB(hipGetLastError());
    VRB(hipStreamSynchronize(st));
    if (c[1] != n - 1) return (int)hipErrorUnknown;  // every interior node allocated exactly once
    *levels = (int)c[2];
    return 0;
}

int device_fill_wide(const Node* bin, const int32_t* desc, uint64_t n4, Node4* out4, void* stream) {
    if (n4 == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(build::fill_wide_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, bin, desc, n4,
                       out4);
    return (int)hipGetLastError();
}

}  // namespace vr

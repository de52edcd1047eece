// vr_host.cpp -- host side of the MI355X path-tracing core: scene construction (copy, the
// reference's median-split BVH build, flattening to the 128-B node layout, HBM upload) and the
// extern "C" entry points declared in include/vanrijn_amd.h.
//
// Reference interfaces replaced here:
//   Scene { camera_location, objects }            src/scene.rs:5-8
//   BoundingVolumeHierarchy::build                src/raycasting/bounding_volume_hierarchy.rs:38-74
//   Plane::new                                    src/raycasting/plane.rs:18-31
//   partial_render_scene                          src/camera.rs:95-130
//   AccumulationBuffer::{new, update_pixel}       src/accumulation_buffer.rs:14-60
//   Spectrum::reflection_from_linear_rgb / intensity_at_wavelength   src/colour/spectrum.rs:64-165
//   ColourXyz::for_wavelength                     src/colour/colour_xyz.rs:22-29, 86-103
//   load_obj                                      src/mesh.rs:13-88
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/vanrijn_amd.h"
#include "rgb_spectrum_tables.h"
#include "vr_layout.h"

#include <zlib.h>

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define VR_HIP(call)                                                                               \
    do {                                                                                           \
        hipError_t e_ = (call);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return fail(VR_ERROR_DEVICE, std::string(#call " failed: ") + hipGetErrorString(e_)); \
    } while (0)

// ------------------------------------------------------------------------------------------
// Host math in the reference's operation order (only what scene setup needs)
// ------------------------------------------------------------------------------------------
struct H3 {
    double x, y, z;
};
double hdot(H3 a, H3 b) {
    double s = -0.0;  // `Sum for f64` folds from -0.0 (vec3.rs:76-82)
    s = s + a.x * b.x;
    s = s + a.y * b.y;
    s = s + a.z * b.z;
    return s;
}
H3 hcross(H3 a, H3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
H3 hnormalize(H3 a) {
    double inv = 1.0 / std::sqrt(hdot(a, a));
    return {a.x * inv, a.y * inv, a.z * inv};
}

// ------------------------------------------------------------------------------------------
// BVH build (bounding_volume_hierarchy.rs:30-74) and flattening
// ------------------------------------------------------------------------------------------
struct Interval {  // util/interval.rs
    double min, max;
};
Interval iv_empty() { return {INFINITY, -INFINITY}; }
bool iv_is_empty(Interval a) { return a.min > a.max; }
Interval iv_union(Interval a, Interval b) {  // interval.rs:66-77 (f64::min/max ignore NaN)
    if (iv_is_empty(a)) return b;
    if (iv_is_empty(b)) return a;
    return {std::fmin(a.min, b.min), std::fmax(a.max, b.max)};
}
Interval iv_expand(Interval a, double v) {  // interval.rs:79-87
    if (iv_is_empty(a)) return {v, v};
    return {std::fmin(a.min, v), std::fmax(a.max, v)};
}
struct Box3 {
    Interval b[3];
};
Box3 box_empty() { return {{iv_empty(), iv_empty(), iv_empty()}}; }
Box3 box_union(const Box3& a, const Box3& b) {
    return {{iv_union(a.b[0], b.b[0]), iv_union(a.b[1], b.b[1]), iv_union(a.b[2], b.b[2])}};
}
int largest_dimension(const Box3& bb) {  // util/axis_aligned_bounding_box.rs:76-99
    int acc = 0;
    double acc_size = 0.0;
    for (int i = 0; i < 3; ++i) {
        double size = bb.b[i].min == bb.b[i].max ? -1.0 : bb.b[i].max - bb.b[i].min;
        if (size > acc_size) {
            acc = i;
            acc_size = size;
        }
    }
    return acc;
}
void box_to_layout(const Box3& bb, double out[6]) {
    for (int i = 0; i < 3; ++i) {
        out[2 * i] = bb.b[i].min;
        out[2 * i + 1] = bb.b[i].max;
    }
}

struct BuildPrim {
    Box3 box;
    double centre[3];
    uint64_t orig;
};

struct BvhBuilder {
    std::vector<BuildPrim> prims;  // permuted in place into leaf order
    std::vector<vr::Node> nodes;   // interior nodes, preorder
    int max_depth = 0;
    int tri_base = 0;

    // Returns the child encoding of the subtree over prims[lo, hi): >= 0 interior node index,
    // < 0 leaf ~(tri_base + leaf position).  `bounds` receives the subtree's box.
    int32_t build(uint64_t lo, uint64_t hi, int level, Box3& bounds) {
        max_depth = std::max(max_depth, level + 1);
        bounds = box_empty();
        for (uint64_t i = lo; i < hi; ++i) bounds = box_union(bounds, prims[i].box);
        if (hi - lo <= 1) return ~(int32_t)(tri_base + lo);
        const int axis = largest_dimension(bounds);
        // sort_unstable_by(centre[axis].partial_cmp, NaN -> Equal); equal keys ordered by input
        // index so the permutation is unique (the oracle applies the same rule)
        std::sort(prims.begin() + lo, prims.begin() + hi, [axis](const BuildPrim& a, const BuildPrim& b) {
            double ca = a.centre[axis], cb = b.centre[axis];
            if (ca < cb) return true;
            if (ca > cb) return false;
            return a.orig < b.orig;
        });
        const uint64_t pivot = (hi - lo) / 2;
        const int32_t me = (int32_t)nodes.size();
        nodes.emplace_back();
        Box3 lb, rb;
        int32_t l = build(lo, lo + pivot, level + 1, lb);
        int32_t r = build(lo + pivot, hi, level + 1, rb);
        vr::Node& n = nodes[me];
        std::memset(&n, 0, sizeof n);
        box_to_layout(lb, n.box[0]);
        box_to_layout(rb, n.box[1]);
        n.child[0] = l;
        n.child[1] = r;
        return me;
    }
};

#ifndef VR_SAH_BINS  // bins per axis of the host's binned SAH (the device build uses 32)
#define VR_SAH_BINS 32
#endif
// Traversal tree (the default): a binned-SAH binary tree over the same triangles, leaf size 1.
// The reference's closest hit does not depend on its tree: a box test on a superset box passes
// whenever it passes on the subset (every rounding step of (bound - o) / d is monotonic in
// `bound`), so a triangle is reachable in the reference tree iff the exact line test passes on
// its OWN box -- which this tree tests too, as the leaf child's box -- and distance ties are
// broken by the reference in-order rank carried in TriVerts::rank.  Only the amount of work
// depends on the tree: SAH splits cut node visits against the median split.
struct SahBuilder {
    std::vector<BuildPrim>& prims;  // permuted in place into this tree's leaf order
    std::vector<vr::Node> nodes;
    int max_depth = 0;
    int tri_base = 0;
    explicit SahBuilder(std::vector<BuildPrim>& p) : prims(p) {}

    static double area(const Box3& b) {
        const double dx = b.b[0].max - b.b[0].min, dy = b.b[1].max - b.b[1].min, dz = b.b[2].max - b.b[2].min;
        if (!(dx >= 0.0) || !(dy >= 0.0) || !(dz >= 0.0)) return 0.0;
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }

    uint64_t split(uint64_t lo, uint64_t hi, int level) {
        const uint64_t n = hi - lo;
        double cmin[3] = {INFINITY, INFINITY, INFINITY}, cmax[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint64_t i = lo; i < hi; ++i)
            for (int c = 0; c < 3; ++c) {
                cmin[c] = std::min(cmin[c], prims[i].centre[c]);
                cmax[c] = std::max(cmax[c], prims[i].centre[c]);
            }
        constexpr int kBins = VR_SAH_BINS;
        int best_axis = -1, best_bin = -1;
        double best_cost = INFINITY;
        // median splits where SAH would push the tree past the deepest traversal stack (48)
        const int need = n > 1 ? 64 - __builtin_clzll(n - 1) : 0;  // ceil(log2 n)
        if (level + need < 44) {
            for (int a = 0; a < 3; ++a) {
                const double ext = cmax[a] - cmin[a];
                if (!(ext > 0.0)) continue;
                Box3 bb[kBins];
                uint64_t cnt[kBins] = {};
                for (int k = 0; k < kBins; ++k) bb[k] = box_empty();
                const double scale = kBins / ext;
                for (uint64_t i = lo; i < hi; ++i) {
                    int k = (int)((prims[i].centre[a] - cmin[a]) * scale);
                    k = std::min(kBins - 1, std::max(0, k));
                    ++cnt[k];
                    bb[k] = box_union(bb[k], prims[i].box);
                }
                double right_area[kBins];
                uint64_t right_cnt[kBins];
                Box3 acc = box_empty();
                uint64_t c = 0;
                for (int k = kBins - 1; k > 0; --k) {
                    acc = box_union(acc, bb[k]);
                    c += cnt[k];
                    right_area[k] = area(acc);
                    right_cnt[k] = c;
                }
                acc = box_empty();
                c = 0;
                for (int k = 0; k < kBins - 1; ++k) {
                    acc = box_union(acc, bb[k]);
                    c += cnt[k];
                    if (c == 0 || right_cnt[k + 1] == 0) continue;
                    const double cost = area(acc) * (double)c + right_area[k + 1] * (double)right_cnt[k + 1];
                    if (cost < best_cost) {
                        best_cost = cost;
                        best_axis = a;
                        best_bin = k;
                    }
                }
            }
        }
        if (best_axis >= 0) {
            const double ext = cmax[best_axis] - cmin[best_axis], scale = kBins / ext;
            auto mid = std::partition(prims.begin() + lo, prims.begin() + hi, [&](const BuildPrim& p) {
                int k = (int)((p.centre[best_axis] - cmin[best_axis]) * scale);
                k = std::min(kBins - 1, std::max(0, k));
                return k <= best_bin;
            });
            const uint64_t m = (uint64_t)(mid - prims.begin());
            if (m > lo && m < hi) return m;
        }
        // median split on the widest centroid axis (ties by reference rank: deterministic)
        int a = 0;
        for (int c = 1; c < 3; ++c)
            if (cmax[c] - cmin[c] > cmax[a] - cmin[a]) a = c;
        const uint64_t m = lo + n / 2;
        std::nth_element(prims.begin() + lo, prims.begin() + m, prims.begin() + hi,
                         [a](const BuildPrim& x, const BuildPrim& y) {
                             if (x.centre[a] < y.centre[a]) return true;
                             if (x.centre[a] > y.centre[a]) return false;
                             return x.orig < y.orig;
                         });
        return m;
    }

    int32_t build(uint64_t lo, uint64_t hi, int level, Box3& bounds) {
        max_depth = std::max(max_depth, level + 1);
        bounds = box_empty();
        for (uint64_t i = lo; i < hi; ++i) bounds = box_union(bounds, prims[i].box);
        if (hi - lo <= 1) return ~(int32_t)(tri_base + lo);
        const uint64_t mid = split(lo, hi, level);
        const int32_t me = (int32_t)nodes.size();
        nodes.emplace_back();
        Box3 lb, rb;
        const int32_t l = build(lo, mid, level + 1, lb);
        const int32_t r = build(mid, hi, level + 1, rb);
        vr::Node& nd = nodes[me];
        std::memset(&nd, 0, sizeof nd);
        box_to_layout(lb, nd.box[0]);
        box_to_layout(rb, nd.box[1]);
        nd.child[0] = l;
        nd.child[1] = r;
        return me;
    }
};

// f32 copies of f64 box bounds, rounded outward (a lower bound down, an upper bound up), so an
// f32 box contains its f64 box
float round_lower(double v) {
    float f = (float)v;
    if ((double)f > v) f = std::nextafter(f, -INFINITY);
    return f;
}
float round_upper(double v) {
    float f = (float)v;
    if ((double)f < v) f = std::nextafter(f, INFINITY);
    return f;
}


// The render kernel's 4-wide tree, collapsed from a binary tree (the SAH traversal tree, or the
// reference's median-split tree): starting from a binary node's two children, the interior child
// with the largest surface area is replaced by its two children until there are four (or only
// leaves).  Leaf children keep the triangle's own box, so DESIGN.md section 5's argument carries
// over unchanged: interior boxes are unions (supersets), and a triangle is tested iff the exact
// line test passes on its own box.  `stack` is the deepest the kernel's traversal stack can get
// (a visit pushes all but one hit interior child): the maximum over root-to-node paths of the
// sum of (interior children - 1).
struct WideBuilder {
    const std::vector<vr::Node>& bin;
    std::vector<vr::Node4>& n4;
    int stack = 0;
    bool dp = false;  // the SAH-optimal DP collapse (else greedy by largest child area)
    WideBuilder(const std::vector<vr::Node>& b, std::vector<vr::Node4>& a, bool dp_ = false) : bin(b), n4(a), dp(dp_) {}

    static double area(const double* b) {
        const double dx = b[1] - b[0], dy = b[3] - b[2], dz = b[5] - b[4];
        if (!(dx >= 0.0) || !(dy >= 0.0) || !(dz >= 0.0)) return 0.0;
        return dx * dy + dy * dz + dz * dx;
    }

    // SAH-optimal collapse (the default; VR_SCENE_GREEDY_COLLAPSE builds the greedy one): a visit of a wide node costs one node step whatever its
    // children, and is entered with probability ~ its surface area, so the wide tree minimising
    // sum(SA(wide node)) is chosen by a bottom-up DP over the binary tree (as in Ylitie et al.'s
    // wide-BVH collapse, leaf size 1): F(x) = SA(x) + H(x, 4) is x as a wide node; C(x, k), the best
    // cost of x's subtree in at most k slots of its parent, = min(F(x), H(x, k)) for k >= 2 (x
    // dissolved into its children) and F(x) for k = 1; H(x, k) = min over a of C(l, a) + C(r, k - a),
    // a leaf costing 0.  split[x][k]: 0 keeps x as one slot, a > 0 gives its left child a slots.
    std::vector<std::array<double, 5>> C;
    std::vector<std::array<uint8_t, 5>> split;
    double H(int32_t x, int k, uint8_t& arg) const {
        double best = INFINITY;
        for (int a = 1; a < k; ++a) {
            const int32_t l = bin[x].child[0], r = bin[x].child[1];
            const double v = (l >= 0 ? C[l][a] : 0.0) + (r >= 0 ? C[r][k - a] : 0.0);
            if (v < best) {
                best = v;
                arg = (uint8_t)a;
            }
        }
        return best;
    }
    void plan(int32_t x, double sa) {  // x interior, sa: its surface area
        if (C.size() < bin.size()) {
            C.resize(bin.size());
            split.resize(bin.size());
        }
        for (int c = 0; c < 2; ++c)
            if (bin[x].child[c] >= 0) plan(bin[x].child[c], area(bin[x].box[c]));
        uint8_t a4 = 1;
        const double f = sa + H(x, 4, a4);
        C[x][1] = f;
        split[x][1] = 0;
        for (int k = 2; k <= 4; ++k) {
            uint8_t a = 1;
            const double h = H(x, k, a);
            C[x][k] = h < f ? h : f;
            split[x][k] = h < f ? a : 0;
        }
        split[x][0] = a4;  // the split of x's two children over a wide node's 4 slots
    }
    void plan_root(int32_t b) {  // before collapse(b, 0) of a BVH root
        double u[6];
        for (int j = 0; j < 6; ++j)
            u[j] = (j & 1) ? std::max(bin[b].box[0][j], bin[b].box[1][j]) : std::min(bin[b].box[0][j], bin[b].box[1][j]);
        plan(b, area(u));
    }
    void expand(int32_t x, const double* bx, int k, int32_t* code, const double** box, int& n) const {
        if (x < 0 || k == 1 || split[x][k] == 0) {
            code[n] = x;
            box[n] = bx;
            ++n;
            return;
        }
        expand(bin[x].child[0], bin[x].box[0], split[x][k], code, box, n);
        expand(bin[x].child[1], bin[x].box[1], k - split[x][k], code, box, n);
    }

    // wide node over binary interior node `b`; `pushed`: stack entries held by its ancestors
    // the children of a wide node over binary node b: the DP's expansion or the greedy one
    int children(int32_t b, bool use_dp, int32_t* code, const double** box) const {
        int n = 0;
        if (use_dp) {
            const int a = split[b][0];
            expand(bin[b].child[0], bin[b].box[0], a, code, box, n);
            expand(bin[b].child[1], bin[b].box[1], 4 - a, code, box, n);
            return n;
        }
        for (int c = 0; c < 2; ++c) {
            code[c] = bin[b].child[c];
            box[c] = bin[b].box[c];
        }
        n = 2;
        while (n < 4) {
            int pick = -1;
            double best = -1.0;
            for (int k = 0; k < n; ++k)
                if (code[k] >= 0 && area(box[k]) > best) {
                    best = area(box[k]);
                    pick = k;
                }
            if (pick < 0) break;
            const vr::Node& c = bin[code[pick]];
            code[pick] = c.child[0];
            box[pick] = c.box[0];
            code[n] = c.child[1];
            box[n] = c.box[1];
            ++n;
        }
        return n;
    }
    // stack bound of the wide subtree over b when every node below uses the DP (or the greedy)
    // expansion: (interior children - 1) + the deepest child's (memoised)
    std::vector<int16_t> need_memo[2];
    int need(int32_t b, bool use_dp) {
        auto& m = need_memo[use_dp];
        if (m.size() < bin.size()) m.assign(bin.size(), -1);
        if (m[b] >= 0) return m[b];
        int32_t code[4];
        const double* box[4];
        const int n = children(b, use_dp, code, box);
        int interior = 0, deepest = 0;
        for (int k = 0; k < n; ++k)
            if (code[k] >= 0) {
                ++interior;
                deepest = std::max(deepest, need(code[k], use_dp));
            }
        return m[b] = (int16_t)(std::max(0, interior - 1) + deepest);
    }
    int limit = 1 << 30;  // dp: a node takes the DP expansion only if its DP subtree's stack fits

    // wide node over binary interior node `b`; `pushed`: stack entries held by its ancestors
    int32_t collapse(int32_t b, int pushed) {
        int32_t code[4];
        const double* box[4];
        // the DP expansion where its whole subtree's stack bound fits under `limit` from here (then
        // it fits at every node below too); else greedy here, and the children decide for themselves
        const int n = children(b, dp && pushed + need(b, true) <= limit, code, box);
        const int32_t me = (int32_t)n4.size();
        n4.emplace_back();
        int interior = 0;
        for (int k = 0; k < n; ++k) interior += code[k] >= 0;
        const int here = pushed + std::max(0, interior - 1);
        stack = std::max(stack, here);
        int32_t out[4];
        for (int k = 0; k < 4; ++k) out[k] = vr::kEmptyChild;
        for (int k = 0; k < n; ++k) out[k] = code[k] >= 0 ? collapse(code[k], here) : code[k];
        vr::Node4& w = n4[me];
        std::memset(&w, 0, sizeof w);
        for (int k = 0; k < 4; ++k) {
            w.child[k] = out[k];
            for (int j = 0; j < 6; ++j) {
                const double v = k < n ? box[k][j] : NAN;
                w.box[k][j] = k < n ? ((j & 1) ? round_upper(v) : round_lower(v)) : NAN;
            }
        }
        return me;
    }
};

// The 4-wide tree over a device-built (median-split) binary tree, planned on the host from the
// triangle count alone: that tree's shape depends only on n (a node over n leaves splits n/2 :
// n - n/2; pre-order indices, the left subtree's m leaves take m - 1 indices), so no node has to
// come back from the device.  Parity collapse: one wide node per binary node at even depth, its
// children the binary node's children or, for interior ones, their two children.  desc: per wide
// node the four slots' box sources (binary node * 2 + child, -1 empty) then their child links;
// vr_build.hip's fill_wide_kernel gathers the boxes.
struct ShapeWide {
    std::vector<int32_t> desc;
    int stack = 0;
    int32_t tri_base = 0;
    struct Sub {
        uint64_t lo, hi;
        int32_t idx;  // global binary index when hi - lo >= 2
    };
    static void kids(const Sub& p, Sub out[2]) {
        const uint64_t mid = p.lo + (p.hi - p.lo) / 2;
        out[0] = {p.lo, mid, p.idx + 1};
        out[1] = {mid, p.hi, p.idx + (int32_t)(mid - p.lo)};
    }
    int32_t wide(const Sub& b, int pushed) {
        const int32_t me = (int32_t)(desc.size() / 8);
        desc.resize(desc.size() + 8, -1);
        int32_t src[4];
        Sub sub[4];
        int n = 0;
        Sub c[2];
        kids(b, c);
        for (int i = 0; i < 2; ++i) {
            if (c[i].hi - c[i].lo == 1) {
                src[n] = b.idx * 2 + i;
                sub[n++] = c[i];
            } else {
                Sub g[2];
                kids(c[i], g);
                for (int j = 0; j < 2; ++j) {
                    src[n] = c[i].idx * 2 + j;
                    sub[n++] = g[j];
                }
            }
        }
        int interior = 0;
        for (int k = 0; k < n; ++k) interior += sub[k].hi - sub[k].lo > 1;
        const int here = pushed + std::max(0, interior - 1);
        stack = std::max(stack, here);
        for (int k = 0; k < 4; ++k) {
            int32_t code = vr::kEmptyChild;
            if (k < n)
                code = sub[k].hi - sub[k].lo == 1 ? ~(tri_base + (int32_t)sub[k].lo) : wide(sub[k], here);
            desc[(size_t)me * 8 + k] = k < n ? src[k] : -1;
            desc[(size_t)me * 8 + 4 + k] = code;
        }
        return me;
    }
};

}  // namespace

// ------------------------------------------------------------------------------------------
// Scene
// ------------------------------------------------------------------------------------------
struct vr_scene {
    int device = -1;
    bool host_only = false;
    double camera[3];
    double extent = 0.0;
    std::vector<vr::Material> materials;
    std::vector<vr::Prim> prims;
    std::vector<vr::Bvh> bvhs;
    std::vector<double> light_dirs;  // Whitted: 3 per light
    std::vector<vr::Node> nodes;
    std::vector<vr::Node4> nodes4;  // the render kernel's 4-wide tree (collapse_wide)
    int wide_stack = 0;             // deepest traversal stack of the 4-wide tree
    uint64_t wide_count = 0;        // its node count
    std::vector<vr::TriVerts> tris;
    std::vector<vr::TriNormals> normals;
    std::vector<std::vector<uint64_t>> leaf_order;  // per mesh
    std::vector<int> mesh_tri_base;
    int max_depth = 0;
    uint32_t object_count = 0;
    // VR_SCENE_DEVICE_BVH: the meshes' BVHs are built on the device after upload (host vectors
    // nodes / tris / normals stay empty; the counts below size the device arrays)
    bool device_bvh = false;
    bool device_sah = false;  // VR_SCENE_DEVICE_SAH: the SAH traversal tree too (vr_build.hip)
    bool greedy_collapse = false;  // VR_SCENE_GREEDY_COLLAPSE: the 4-wide tree by largest child area
    bool force_big = false;        // VR_SCENE_WIDE_OFFSETS: the 64-bit-offset kernels for any size
    uint64_t staging_limit = 0;    // vr_scene_set_staging_limit: bytes of staging per call (0: half the free HBM)
    uint64_t node_count = 0, tri_count = 0;
    struct PendingMesh {
        const double* vertices;
        const double* normals;
        uint64_t n;
        int32_t node_base, tri_base;
        uint32_t mesh;
    };
    std::vector<PendingMesh> pending;
    bool dark0 = true;  // every material's colour(0 nm) == 0: the recursion-limit photon needs no lambda-0 chain
    int mats = 0;       // bit 0: a Lambertian material exists, bit 1: a reflective one
    // every continuation of every path yields a finite intensity (shading_finite on each traced
    // mesh, no Phong or dielectric material): then a path with zero throughput may stop early and
    // the recursion-limit lambda-0 chain may be taken as b0 (DARK0); otherwise both are traced so
    // that a later NaN reaches the photon as in the reference (0 * NaN)
    bool nan_free = true;
    // device copies
    void* d_block = nullptr;
    size_t device_bytes = 0;
    vr::DeviceScene dev{};
    unsigned long long* d_counters = nullptr;
    std::mutex counter_mutex;
    std::atomic<uint64_t> pass_counter{0};
    // render-call contexts (stream, staging buffer, work-queue counter, error word, scratch),
    // pooled: concurrent calls each hold their own, so they neither share a staging buffer nor
    // read each other's error word (include/vanrijn_amd.h "Threading")
    std::mutex ctx_mutex;
    std::vector<struct CallCtx*> ctx_all, ctx_free;
    // sticky per-stream error words of the asynchronous entry point (vr_render_tile_device),
    // read and cleared by vr_stream_check_error or a timed launch on that stream
    std::mutex slot_mutex;
    std::unordered_map<void*, int32_t*> stream_slots;
    // deferred launch timings (VR_LAUNCH_DEFER_TIMES), per stream, under slot_mutex: the HIP events
    // of launches not yet read by vr_collect_launch_times -- [start, mid, end] per pass -- and the
    // passes of each launch
    struct Deferred {
        std::vector<hipEvent_t> ev;
        std::vector<uint32_t> passes;
    };
    std::unordered_map<void*, Deferred> deferred;
    int cu_count = 0;
    uint64_t partial_seed = 0x5EED0001ull;
    // test hook (vr_debug_set_fault_object): hits on this object take the singular-basis path,
    // which finite geometry cannot reach (DESIGN.md "Errors")
    int32_t fault_object = -1;
    // test hook (vr_debug_set_launch_flags): launch flags OR'ed into every render of the scene
    uint32_t debug_launch_flags = 0;
};

// The render kernel addresses the triangle and 4-wide node arrays with 32-bit byte offsets from
// their scalar bases (tri * 80, node << 7); a scene past either limit -- 53.7 M triangles (4 GB of
// TriVerts), 2^25 wide nodes -- runs the kernels with 64-bit offsets (render_kernel<.., BIG>)
static bool needs_big_offsets(uint64_t tri_count, uint64_t wide_count) {
    return tri_count * sizeof(vr::TriVerts) >= (1ull << 32) || wide_count >= (1ull << 25);
}
static bool needs_big_offsets(const vr_scene* s) {
    return s->force_big || needs_big_offsets(s->tri_count, s->wide_count);
}

// One render call's device resources.  `done` is recorded on the launch stream after the last
// kernel that reads `staging` / `queue`; a later user of the context waits on it first.
struct CallCtx {
    hipStream_t stream = nullptr;  // the host-buffer entry points' own stream
    hipEvent_t done = nullptr;
    void* staging = nullptr;  // 16 B per (pixel, sample) of a pass
    size_t staging_bytes = 0;
    unsigned long long* queue = nullptr;  // work-item counter; error word at queue + 8
    int32_t* error = nullptr;
    void* scratch = nullptr;  // device records + host-layout buffers of the host-buffer calls
    size_t scratch_bytes = 0;
    void* pinned = nullptr;  // page-locked host copy of the host-layout buffers (DMA at full PCIe rate)
    size_t pinned_bytes = 0;
    void* mask = nullptr;  // camera-frustum culled 8x8 blocks of the call's tile (1 B each)
    size_t mask_bytes = 0;
    hipStream_t last_stream = nullptr;  // the stream of the last call's work (enqueue_passes)
    bool used = false;
    // debug builds (-DVR_STAGE_GUARD): a generation tag beside every staging slot, and the last
    // pass generation this context used
    void* tags = nullptr;
    size_t tag_bytes = 0;
    uint32_t gen = 0;
};

// ---------------------------------------------------------------------------------------------
// Host threads for the host-buffer entry points: copying the AccumulationBuffer arrays between
// page-locked staging and the caller's memory, and vr_merge_tile.  88 B per pixel of host memory
// traffic is ~5 ms per 1024^2 frame on one core -- more than the GPU's share of a 1-spp render.
// ---------------------------------------------------------------------------------------------
// Environment overrides exist in tuning builds only (python -m vanrijn_amd.build with VR_TUNING=1,
// -DVR_TUNING_VARIANTS: tools/variants.py threshold sweeps, tools/cycles.py diagnostics); a default
// build reads no VR_* variable, so nothing in a user's environment changes rendering or timing.
// launch defaults (A/B builds may override them at compile time)
#ifndef VR_COOP_SAMPLES  // launches of at most this many pixel-samples may take the cooperative tail
#define VR_COOP_SAMPLES (4ull << 20)
#endif
#ifndef VR_COOP_BOUNCES  // ... once every live path of a wave has bounced this often
#define VR_COOP_BOUNCES 0u
#endif
static const char* tuning_env(const char* name) {
#ifdef VR_TUNING_VARIANTS
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

// the CPUs this process may run on (sched affinity), at most 16 (VR_HOST_THREADS overrides in
// tuning builds)
static unsigned host_threads() {
    static const unsigned n = [] {
        unsigned c = 0;
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof set, &set) == 0) c = (unsigned)CPU_COUNT(&set);
        if (c == 0) c = std::thread::hardware_concurrency();
        if (const char* e = tuning_env("VR_HOST_THREADS")) c = (unsigned)atoi(e);
        return std::max(1u, std::min(c, 16u));
    }();
    return n;
}

// A persistent pool: run(parts, fn) calls fn(0..parts-1) on the pool's threads and the caller's,
// and returns when all parts are done.  Concurrent callers share the pool (jobs queue FIFO; each
// caller also works on its own job, so a busy pool never blocks progress).
class HostPool {
  public:
    static HostPool& get() {
        static HostPool* p = new HostPool(host_threads() - 1);  // never destroyed: threads idle at exit
        return *p;
    }
    void run(unsigned parts, const std::function<void(unsigned)>& fn) {
        if (parts == 0) return;
        Job j;
        j.fn = &fn;
        j.parts = parts;
        if (parts > 1 && !threads_.empty()) {
            std::lock_guard<std::mutex> g(m_);
            jobs_.push_back(&j);
            cv_.notify_all();
        }
        for (unsigned i; (i = j.next.fetch_add(1)) < parts;) {
            fn(i);
            j.done.fetch_add(1);
        }
        std::unique_lock<std::mutex> l(m_);
        for (auto it = jobs_.begin(); it != jobs_.end(); ++it)
            if (*it == &j) {
                jobs_.erase(it);
                break;
            }
        done_cv_.wait(l, [&] { return j.done.load() == parts; });
    }

  private:
    struct Job {
        const std::function<void(unsigned)>* fn = nullptr;
        unsigned parts = 0;
        std::atomic<unsigned> next{0}, done{0};
    };
    explicit HostPool(unsigned n) {
        for (unsigned i = 0; i < n; ++i) threads_.emplace_back([this] { work(); });
    }
    void work() {
        std::unique_lock<std::mutex> l(m_);
        while (true) {
            cv_.wait(l, [&] { return !jobs_.empty(); });
            Job* j = jobs_.front();
            const unsigned i = j->next.fetch_add(1);
            if (i >= j->parts) {  // every part taken: the job leaves the queue
                jobs_.pop_front();
                continue;
            }
            l.unlock();
            (*j->fn)(i);
            const bool last = j->done.fetch_add(1) + 1 == j->parts;
            l.lock();
            if (last) done_cv_.notify_all();
        }
    }
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    std::deque<Job*> jobs_;
    std::vector<std::thread> threads_;
};

// fn(begin, end) over [0, n) in about `host_threads()` pieces of at least `grain`
static void parallel_range(uint64_t n, uint64_t grain, const std::function<void(uint64_t, uint64_t)>& fn) {
    const uint64_t pieces = std::max<uint64_t>(1, std::min<uint64_t>(host_threads(), n / std::max<uint64_t>(1, grain)));
    if (pieces <= 1) {
        fn(0, n);
        return;
    }
    const uint64_t step = (n + pieces - 1) / pieces;
    HostPool::get().run((unsigned)pieces, [&](unsigned i) {
        const uint64_t b = std::min(n, (uint64_t)i * step), e = std::min(n, b + step);
        if (b < e) fn(b, e);
    });
}

// copy `bytes` in parallel (host memory bandwidth, not one core's)
static void parallel_copy(void* dst, const void* src, size_t bytes) {
    parallel_range(bytes, (size_t)1 << 20, [&](uint64_t b, uint64_t e) {
        std::memcpy((char*)dst + b, (const char*)src + b, e - b);
    });
}

// Whether every hit on this mesh has a finite shading basis, whatever the barycentric point: the
// reference's normal = normalize(sum b_i N_i) (triangle.rs:73-78) is NaN where the interpolated
// normal is zero (mesh.rs:37 gives zero normals to an OBJ without them), and cotangent =
// normalize((V0 - V1) x n) is NaN where n is parallel to that edge.  Sufficient: all three vertex
// normals lie strictly on one side of the triangle's plane, by a relative margin of 1e-6 (then
// n . f >= 1e-6 |N|max |f| sum(b) - O(1e-16), so n is nonzero and not in the plane, where the edge
// lies), with magnitudes far from f64 under- / overflow.  Degenerate triangles fail.  (A sphere's
// basis is NaN only where a hit's x and y equal the centre's exactly, and a retro direction only
// where a hit lies exactly at the ray origin: exact-equality events of measure zero, not excluded.)
static bool shading_finite(const vr_mesh_desc& m) {
    for (uint64_t t = 0; t < m.triangle_count; ++t) {
        const double* v = m.vertices + 9 * t;
        const double* nn = m.normals + 9 * t;
        for (int i = 0; i < 9; ++i)
            if (!std::isfinite(v[i]) || !std::isfinite(nn[i]) || std::fabs(v[i]) > 1e100 || std::fabs(nn[i]) > 1e100)
                return false;
        const double e1[3] = {v[3] - v[0], v[4] - v[1], v[5] - v[2]}, e2[3] = {v[6] - v[0], v[7] - v[1], v[8] - v[2]};
        const double f[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        const double fl = std::sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
        if (!(fl > 1e-200)) return false;
        double nmax = 0.0, d[3];
        for (int k = 0; k < 3; ++k) {
            const double* n = nn + 3 * k;
            nmax = std::max(nmax, std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]));
            d[k] = n[0] * f[0] + n[1] * f[1] + n[2] * f[2];
        }
        if (!(nmax > 1e-100)) return false;
        const double m6 = 1e-6 * nmax * fl;
        if (!((d[0] > m6 && d[1] > m6 && d[2] > m6) || (d[0] < -m6 && d[1] < -m6 && d[2] < -m6))) return false;
    }
    return true;
}

// spectrum.rs:64-79's sample wavelengths as the reference computes them (before / after), and the
// reciprocal step for the device's segment index (intensity only: a neighbouring segment at a knot
// gives the same value to rounding)
static void fill_knots(vr::Material& m) {
    const double range = m.longest - m.shortest;
    for (int j = 0; j < m.n; ++j) m.knots[j] = (double)j / (double)(m.n - 1) * range + m.shortest;
    m.inv_step = m.n > 1 && range > 0.0 ? (double)(m.n - 1) / range : 0.0;
}

namespace {

int stack_depth(const vr_scene* s) { return std::max(1, s->max_depth - 1); }  // binary tree walks
int wide_stack_depth(const vr_scene* s) { return s->wide_stack + 1; }  // render kernel (+1: branchless pushes)


// the render kernel's 4-wide tree over every traversed mesh's binary tree `nodes`
void collapse_wide(vr_scene* s, const std::vector<vr::Node>& nodes) {
    // greedy collapse; unless VR_SCENE_GREEDY_COLLAPSE, the SAH-optimal one instead wherever its (deeper) stack
    // bound keeps the kernel in the greedy tree's LDS stack class (24 / 32 / 48 entries; a larger
    // class would cost workgroups per CU): a node takes the DP expansion when its DP subtree fits
    auto class_limit = [](int st) { return st + 1 <= 24 ? 23 : (st + 1 <= 32 ? 31 : 47); };
    std::vector<vr::Node4> greedy;
    WideBuilder G(nodes, greedy, false);
    std::vector<int32_t> groot(s->bvhs.size());
    for (size_t i = 0; i < s->bvhs.size(); ++i)
        groot[i] = s->bvhs[i].root >= 0 ? G.collapse(s->bvhs[i].root, 0) : s->bvhs[i].root;
    bool use_dp = false;
    std::vector<vr::Node4> opt;
    std::vector<int32_t> oroot(s->bvhs.size());
    int ostack = 0;
    if (!s->greedy_collapse) {
        WideBuilder D(nodes, opt, true);
        D.limit = class_limit(G.stack);
        for (size_t i = 0; i < s->bvhs.size(); ++i) {
            if (s->bvhs[i].root >= 0) D.plan_root(s->bvhs[i].root);
            oroot[i] = s->bvhs[i].root >= 0 ? D.collapse(s->bvhs[i].root, 0) : s->bvhs[i].root;
        }
        ostack = D.stack;
        use_dp = D.stack <= D.limit;  // (by construction)
    }
    s->nodes4 = use_dp ? std::move(opt) : std::move(greedy);
    for (size_t i = 0; i < s->bvhs.size(); ++i) s->bvhs[i].root4 = use_dp ? oroot[i] : groot[i];
    s->wide_stack = use_dp ? ostack : G.stack;
    s->wide_count = s->nodes4.size();
    if (tuning_env("VR_WIDE_STATS")) {  // diagnostic: the collapse's SAH objective, sum SA(wide) / SA(root)
        double sum = 0.0, root = 0.0;
        for (const auto& w : s->nodes4) {
            float u[6] = {INFINITY, -INFINITY, INFINITY, -INFINITY, INFINITY, -INFINITY};
            for (int k = 0; k < 4; ++k)
                if (w.child[k] != vr::kEmptyChild)
                    for (int j = 0; j < 6; ++j) u[j] = (j & 1) ? std::max(u[j], w.box[k][j]) : std::min(u[j], w.box[k][j]);
            const double a = (double)(u[1] - u[0]) * (u[3] - u[2]) + (double)(u[3] - u[2]) * (u[5] - u[4]) +
                             (double)(u[5] - u[4]) * (u[1] - u[0]);
            sum += a;
            if (&w == &s->nodes4[0]) root = a;
        }
        std::fprintf(stderr, "vr wide tree: %zu nodes, stack %d, sum SA / SA(first root) %.4f (%s collapse)\n",
                     s->nodes4.size(), s->wide_stack, sum / root, use_dp ? "DP" : "greedy");
    }
}

template <class T>
size_t align_up(size_t v) {
    return (v + 255) & ~size_t(255);
}

struct CallScratch {
    hipStream_t stream = nullptr;
    void* ptr = nullptr;
    ~CallScratch() {
        if (ptr) (void)hipFree(ptr);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

int upload(vr_scene* s) {
    VR_HIP(hipSetDevice(s->device));
    const size_t sz_nodes = s->node_count * sizeof(vr::Node);
    // the 4-wide tree has at most one node per binary interior node (device builds collapse after
    // the build, so its arrays are sized by that bound)
    const size_t sz_nodes4 = s->node_count * sizeof(vr::Node4);
    const size_t sz_tris = s->tri_count * sizeof(vr::TriVerts);
    const size_t sz_norm = s->tri_count * sizeof(vr::TriNormals);
    const size_t sz_mat = s->materials.size() * sizeof(vr::Material);
    const size_t sz_prim = s->prims.size() * sizeof(vr::Prim);
    const size_t sz_bvh = s->bvhs.size() * sizeof(vr::Bvh);
    size_t off[8], total = 0;
    const size_t sz_misc = 64 + vr::kCntCount * sizeof(unsigned long long);  // error flag, counters
    const size_t sizes[8] = {sz_nodes, sz_tris, sz_norm, sz_mat, sz_prim, sz_bvh,
                             sz_misc + 3 * VR_MAX_LIGHTS * sizeof(double), sz_nodes4};
    for (int i = 0; i < 8; ++i) {
        off[i] = total;
        total += align_up<char>(std::max<size_t>(sizes[i], 1));
    }
    VR_HIP(hipMalloc(&s->d_block, total));
    s->device_bytes = total;
    VR_HIP(hipDeviceGetAttribute(&s->cu_count, hipDeviceAttributeMultiprocessorCount, s->device));
    char* base = (char*)s->d_block;
    const void* src[6] = {s->nodes.data(), s->tris.data(), s->normals.data(), s->materials.data(), s->prims.data(),
                          s->bvhs.data()};
    for (int i = 0; i < 6; ++i) {
        if (s->device_bvh && (i < 3 || i == 5)) continue;  // filled by the device build below
        if (sizes[i]) VR_HIP(hipMemcpy(base + off[i], src[i], sizes[i], hipMemcpyHostToDevice));
    }
    VR_HIP(hipMemset(base + off[6], 0, sizes[6]));
    s->d_counters = (unsigned long long*)(base + off[6] + 64);
    s->dev.light_dirs = (const double*)(base + off[6] + sz_misc);
    if (!s->light_dirs.empty())
        VR_HIP(hipMemcpy(base + off[6] + sz_misc, s->light_dirs.data(), s->light_dirs.size() * sizeof(double),
                         hipMemcpyHostToDevice));
    vr::DeviceScene& d = s->dev;
    d.nodes = (const vr::Node*)(base + off[0]);
    d.nodes4 = (const vr::Node4*)(base + off[7]);
    d.tris = (const vr::TriVerts*)(base + off[1]);
    d.normals = (const vr::TriNormals*)(base + off[2]);
    d.materials = (const vr::Material*)(base + off[3]);
    d.prims = (const vr::Prim*)(base + off[4]);
    d.bvhs = (const vr::Bvh*)(base + off[5]);
    if (s->device_bvh) {
        // BoundingVolumeHierarchy::build on the device (vr_build.hip): same nodes, same leaf order
        CallScratch cs;
        VR_HIP(hipStreamCreateWithFlags(&cs.stream, hipStreamNonBlocking));
        vr::Node* nodes = (vr::Node*)(base + off[0]);
        for (const auto& pm : s->pending) {
            double root_box[6];
            int levels = 0;
            const int e = vr::device_build_bvh(pm.vertices, pm.normals, (uint32_t)pm.n, pm.node_base, pm.tri_base,
                                               nodes + pm.node_base, (vr::TriVerts*)(base + off[1]) + pm.tri_base,
                                               (vr::TriNormals*)(base + off[2]) + pm.tri_base,
                                               s->leaf_order[pm.mesh].data(), root_box, &levels, cs.stream);
            if (e) return fail(VR_ERROR_DEVICE, std::string("device BVH build failed: ") +
                                                    hipGetErrorString((hipError_t)e));
            s->max_depth = std::max(s->max_depth, levels);
        }
        VR_HIP(hipStreamSynchronize(cs.stream));
        if (s->device_sah && s->device_bvh) {
            // the SAH traversal tree over the ranked triangles (replaces the median tree in the
            // binary array; the triangles move into its leaf order), then the 4-wide collapse on
            // the host's binary copy (WideBuilder: depth-first layout, as the host-built scene)
            for (const auto& pm : s->pending) {
                if (pm.n < 2) continue;
                double root_box[6];
                int levels = 0;
                const int e = vr::device_build_sah((vr::TriVerts*)(base + off[1]) + pm.tri_base,
                                                   (vr::TriNormals*)(base + off[2]) + pm.tri_base, (uint32_t)pm.n,
                                                   pm.node_base, pm.tri_base, nodes + pm.node_base, root_box, &levels,
                                                   cs.stream);
                if (e) return fail(VR_ERROR_DEVICE, std::string("device SAH build failed: ") +
                                                        hipGetErrorString((hipError_t)e));
                s->max_depth = std::max(s->max_depth, levels);
            }
            s->nodes.resize(s->node_count);
            if (s->node_count)
                VR_HIP(hipMemcpy(s->nodes.data(), nodes, s->node_count * sizeof(vr::Node), hipMemcpyDeviceToHost));
            collapse_wide(s, s->nodes);
            s->nodes.clear();
            s->nodes.shrink_to_fit();
            s->pending.clear();
            if (sz_bvh) VR_HIP(hipMemcpy(base + off[5], s->bvhs.data(), sz_bvh, hipMemcpyHostToDevice));
            if (!s->nodes4.empty())
                VR_HIP(hipMemcpy(base + off[7], s->nodes4.data(), s->nodes4.size() * sizeof(vr::Node4),
                                 hipMemcpyHostToDevice));
            s->nodes4.clear();
            s->nodes4.shrink_to_fit();
            return VR_OK;
        }
        // the 4-wide traversal tree: planned from the meshes' sizes (ShapeWide), boxes gathered on
        // the device
        ShapeWide W;
        for (const auto& pm : s->pending) {
            if (pm.n < 2) continue;  // one-triangle mesh: its root is the leaf
            W.tri_base = pm.tri_base;
            const int32_t root = W.wide({0, pm.n, pm.node_base}, 0);
            for (auto& b : s->bvhs)
                if (b.tri_base == pm.tri_base && b.root == pm.node_base) b.root4 = root;
        }
        for (auto& b : s->bvhs)
            if (b.root < 0) b.root4 = b.root;
        s->wide_stack = W.stack;
        s->wide_count = W.desc.size() / 8;
        if (s->wide_count) {
            int32_t* d_desc = nullptr;
            VR_HIP(hipMalloc(&d_desc, W.desc.size() * sizeof(int32_t)));
            const hipError_t ec = hipMemcpy(d_desc, W.desc.data(), W.desc.size() * sizeof(int32_t), hipMemcpyHostToDevice);
            const int e = ec != hipSuccess ? (int)ec
                                           : vr::device_fill_wide(nodes, d_desc, s->wide_count, (vr::Node4*)(base + off[7]),
                                                                  cs.stream);
            const hipError_t es = hipStreamSynchronize(cs.stream);
            (void)hipFree(d_desc);
            if (e || es != hipSuccess) return fail(VR_ERROR_DEVICE, "device wide-tree fill failed");
        }
        s->pending.clear();  // the caller's arrays are not kept
        if (sz_bvh) VR_HIP(hipMemcpy(base + off[5], s->bvhs.data(), sz_bvh, hipMemcpyHostToDevice));
    }
    if (!s->nodes4.empty()) {
        VR_HIP(hipMemcpy(base + off[7], s->nodes4.data(), s->nodes4.size() * sizeof(vr::Node4), hipMemcpyHostToDevice));
    }
    return VR_OK;
}

int check_render_params(const vr_scene* s, const vr_render_params* p) {
    if (!s || !p) return fail(VR_ERROR_INVALID_ARGUMENT, "null scene or params");
    if (s->host_only) return fail(VR_ERROR_HOST_ONLY, "scene was created with VR_SCENE_HOST_ONLY");
    const vr_tile& t = p->tile;
    // Tile and Array2D index asserts in the reference (array2d.rs:58,65) panic; here: an error
    if (t.end_column < t.start_column || t.end_row < t.start_row || t.end_column > p->width ||
        t.end_row > p->height || p->width == 0 || p->height == 0)
        return fail(VR_ERROR_INVALID_ARGUMENT, "tile outside the image");
    // the random stream's base mix64(key ^ (pixel << 32 | sample)) is injective
    // only for pixel and sample indices below 2^32: a larger index would silently carry into the
    // other field and repeat another (pixel, sample)'s stream
    if (p->width > (1ull << 32) || p->height > (1ull << 32) || p->width * p->height > (1ull << 32))
        return fail(VR_ERROR_UNSUPPORTED, "image of more than 2^32 pixels (random stream index space)");
    if ((uint64_t)p->first_sample + p->spp > (1ull << 32) || (uint64_t)p->first_sample >= (1ull << 32))
        return fail(VR_ERROR_UNSUPPORTED, "sample indices past 2^32 (random stream index space)");
    if (stack_depth(s) > 48 || wide_stack_depth(s) > 48)
        return fail(VR_ERROR_UNSUPPORTED, "BVH deeper than the largest traversal stack (48)");
    return VR_OK;
}

// persistent grid: workgroups per CU of the render kernel (3: 3 waves per SIMD); VR_GRID_PER_CU
// overrides (tuning builds; diagnostic: throughput against occupancy)
int grid_per_cu() {
    const char* g = tuning_env("VR_GRID_PER_CU");
    return g ? std::max(1, atoi(g)) : 3;
}
// ... of the cooperative-tail instantiations.  They run at VR_COOP_MINW = 2 waves per SIMD, so only 2
// workgroups per CU are resident; the third starts as another retires.  Kept on purpose:
// C1 1.558 ms at 3 per CU against 1.572-1.604 at 2 (9 interleaved repetitions each,
// profiles/r06/probe/coopgrid.out) -- a late-starting workgroup takes items the resident ones would
// otherwise have taken in their tails
int coop_grid_per_cu() {
    const char* g = tuning_env("VR_COOP_GRID");
    return g ? std::max(1, atoi(g)) : 3;
}

#ifdef VR_SPLIT_PROBE  // analysis builds: the ray dump every render launch appends to (vr_probe_set_dump)
struct {
    double* rays;
    unsigned long long* count;
    uint64_t cap;
} g_probe = {nullptr, nullptr, 0};
#endif

vr::RenderArgs make_args(const vr_scene* s, const vr_render_params* p, double* state) {
    vr::RenderArgs a{};
    a.scene = s->dev;
    a.start_column = p->tile.start_column;
    a.start_row = p->tile.start_row;
    a.tile_width = p->tile.end_column - p->tile.start_column;
    a.tile_height = p->tile.end_row - p->tile.start_row;
    a.width = p->width;
    a.height = p->height;
    a.seed = p->seed;
#ifdef VR_SPLIT_PROBE
    a.probe_rays = g_probe.rays;
    a.probe_count = g_probe.count;
    a.probe_n = g_probe.cap;
#endif
    {  // vr-hash32 v2: the launch-constant key of stream_base_keyed
        uint64_t z = p->seed ^ 0x76616E52696A6E31ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        a.seed_key = z ^ (z >> 31);
    }
    a.first_sample = p->first_sample;
    a.spp = p->spp;
    a.accumulate = p->accumulate;
    a.state = state;
    a.records = nullptr;
    a.counters = nullptr;
    a.wg_times = nullptr;
    a.error_flag = nullptr;  // per call (enqueue_passes)
    a.block_mask = nullptr;  // per call (enqueue_passes)
    a.live_blocks = nullptr;
    a.live_count = nullptr;
    a.stage_tag = nullptr;  // debug builds: per call (enqueue_passes)
    a.stage_gen = 0;
    a.pad_gen = 0;
    a.fault_object = s->fault_object;
    const char* th = tuning_env("VR_SHADE_THRESHOLD");  // tuning hook (tools/variants.py)
    a.shade_threshold = th ? (uint32_t)atoi(th) : 52u;
    const char* sm = tuning_env("VR_SHADE_MIN");  // tuning hook: defer shading below this many hits
    a.shade_min = sm ? (uint32_t)std::max(0, atoi(sm)) : 16u;
    a.early_stop = s->nan_free ? 1u : 0u;
    if (const char* es = tuning_env("VR_EARLY_STOP")) a.early_stop = atoi(es) != 0 && s->nan_free;  // A/B hook (off only)
    const char* mm = tuning_env("VR_MISS_MIN");  // tuning hook: defer finishing misses
    a.miss_min = mm ? (uint32_t)std::max(0, atoi(mm)) : 8u;
    const char* ch = tuning_env("VR_CHUNK");  // tuning hook: samples per work item
    a.chunk = ch ? (uint32_t)std::max(1, atoi(ch)) : 1u;
    const char* ts = tuning_env("VR_TAIL_SAMPLES");  // tuning hook: single-sample items at the end
    a.tail_samples = ts ? (uint32_t)std::max(0, atoi(ts)) : 0u;
    const char* gr = tuning_env("VR_GRAB");  // tuning hook: items per queue atomic
    if (gr) {
        a.grab = (uint32_t)std::max(0, atoi(gr));
    } else {
        // 512 items per atomic keeps the queue counter cold on full frames; a smaller launch would
        // hand 512 items to a few waves and leave the rest of the chip idle at its end (1 spp of
        // 1024^2: 1.9 ms at 512), so every wave gets about 80 slices, in multiples of 64 (one item
        // per lane), and at least 128: one atomic per 64 items costs more than the tail it saves.
        // Measured (1024^2): 256 spp best at 512 (64: +38 %, 256: +0.3 %), 64 spp at 256 (512:
        // +1.5 %), C5's mesh at 32 spp at 128; 512^2 @64 (C2) 128..384 within 2 % (64: +17 %);
        // 256^2 @16 (C1) flat (profiles/r02/sweeps/sw_grab_*.txt)
        const uint64_t items = ((a.tile_width + 7) / 8) * ((a.tile_height + 7) / 8) * 64 * std::max(1u, p->spp);
        const uint64_t waves = (uint64_t)std::max(1, s->cu_count) * 3 * 4;
        const uint64_t g = items / (waves * 80) / 64 * 64;
        a.grab = (uint32_t)std::min<uint64_t>(512, std::max<uint64_t>(128, g));
    }
    const char* lt = tuning_env("VR_LEAF_THRESHOLD");  // tuning hooks
    a.leaf_threshold = lt ? (uint32_t)std::max(1, atoi(lt)) : 48u;
    const char* ls = tuning_env("VR_LEAF_STALL");
    a.leaf_stall = ls ? (uint32_t)std::max(1, atoi(ls)) : 3u;
    const char* lf = tuning_env("VR_LEAF_FEW");  // tuning hook (0: off)
    a.leaf_few = lf ? (uint32_t)std::max(0, atoi(lf)) : 0u;
    // the cooperative tail (vr_render.hip coop_step, the COOP instantiations): launches of at most
    // 4 M pixel-samples (a small frame's time is its longest paths') of scenes with a reflective
    // material (paths trapped between mirror facets run to the 128-bounce limit: C1,
    // benches/simple_scene.rs).  Scenes without mirrors never take it: on main.rs's Lambertian scene
    // the breadth-first walk of short tail paths cost more than it saved.
    {
        const uint64_t lsamples = a.tile_width * a.tile_height * (uint64_t)p->spp;
        // (a.coop: the most live paths a wave's tail may have to start it: coop_step serves one or
        // two, lone_walk's whole walks up to four)
        a.coop = (lsamples <= VR_COOP_SAMPLES && (s->mats & 2) && s->dark0) ? 4u : 0u;
        if (const char* co = tuning_env("VR_COOP")) a.coop = (uint32_t)std::min(4, std::max(0, atoi(co)));
        a.coop_bounces = VR_COOP_BOUNCES;  // ... once every live path of the wave has bounced this often
        a.lone_walk = 1;
        if (const char* cb = tuning_env("VR_COOP_BOUNCES")) a.coop_bounces = (uint32_t)std::max(0, atoi(cb));
    }
    {
        // the node step's child keys keep the entry distance's high bits above the node index:
        // the fewest low bits whose all-ones value exceeds every wide node index
        uint32_t m = 1;
        while (m < s->wide_count + 1 && m != 0xffffffffu) m = m << 1 | 1;
        a.sort_mask = m;
    }
    // block-major work items over the live blocks in Z-order (round 5): the waves in flight share a
    // compact patch of the image, so their camera rays and first hits walk the same part of the
    // tree -- C3 -4.5 %, C2 -4.5 %, C5 -4.2 %; scenes with a reflective material keep sample-major
    // order (the bench scene +1..4 % block-major: its trapped mirror paths cluster in the same waves)
    // (profiles/r05/order)
    const bool block_major = (s->mats & 2) == 0;
    const char* io = tuning_env("VR_ITEM_ORDER");  // tuning hook: 0 sample-major, 1 block-major
    a.item_order = io ? (uint32_t)(atoi(io) != 0) : (block_major ? 1u : 0u);
    const char* pr = tuning_env("VR_PHASE_A_REPS");  // tuning hook
    a.phase_a_reps = pr ? (uint32_t)std::max(1, atoi(pr)) : 2u;
    {
        // same f64 operations as the reference's ImageSampler::new / film_to_world
        const double fw = (double)a.width, fh = (double)a.height;
        const double film_w = fw > fh ? fw / fh : 1.0;
        const double film_h = fw > fh ? 1.0 : fw / fh;
        a.film[0] = film_w * (1.0 / fw);
        a.film[1] = film_w * 0.5;
        a.film[2] = film_h * (1.0 / fh);
        a.film[3] = film_h * 0.5;
    }
    {
        const uint64_t bw = (a.tile_width + 7) / 8, bh = (a.tile_height + 7) / 8;
        a.rcp_blocks = bw * bh ? 1.0 / (double)(bw * bh) : 0.0;
        a.rcp_bw = bw ? 1.0 / (double)bw : 0.0;
    }
    a.queue = nullptr;  // per call (enqueue_passes)
    a.staging = nullptr;
    return a;
}

// Waits for `stream`, then reads and clears one error word (a call's own, or a stream's sticky one).
int read_and_clear_error(int32_t* slot, hipStream_t stream) {
    int32_t flag = 0;
    VR_HIP(hipMemcpyAsync(&flag, slot, sizeof flag, hipMemcpyDeviceToHost, stream));
    VR_HIP(hipStreamSynchronize(stream));
    if (flag) {
        VR_HIP(hipMemsetAsync(slot, 0, sizeof flag, stream));
        VR_HIP(hipStreamSynchronize(stream));
        if (flag & 8)  // debug builds (VR_STAGE_GUARD)
            return fail(VR_ERROR_DEVICE, "staging guard: the ordered reduce read a staged photon its pass did not write");
        return fail(VR_ERROR_SINGULAR_BASIS,
                    "Normal, tangent and cotangent don't form a valid basis (det == 0); the reference panics here");
    }
    return VR_OK;
}

// Grow a context buffer to `need` bytes; its previous contents may still be in use by the
// context's last call (on whatever stream), so wait for `done` before freeing it.
int ctx_grow(void** ptr, size_t* have, size_t need, hipEvent_t done) {
    if (need <= *have) return VR_OK;
    VR_HIP(hipEventSynchronize(done));
    if (*ptr) VR_HIP(hipFree(*ptr));
    *ptr = nullptr;
    *have = 0;
    VR_HIP(hipMalloc(ptr, need));
    *have = need;
    return VR_OK;
}

// Grow the context's page-locked host buffer (its previous contents are only read by the host
// within the call that filled it, so no device wait is needed beyond the context's `done`).
int ctx_grow_pinned(CallCtx* c, size_t need) {
    if (need <= c->pinned_bytes) return VR_OK;
    VR_HIP(hipEventSynchronize(c->done));
    if (c->pinned) VR_HIP(hipHostFree(c->pinned));
    c->pinned = nullptr;
    c->pinned_bytes = 0;
    VR_HIP(hipHostMalloc(&c->pinned, need, hipHostMallocDefault));
    c->pinned_bytes = need;
    return VR_OK;
}

void ctx_free_all(CallCtx* c) {
    if (c->done) {
        (void)hipEventSynchronize(c->done);
        (void)hipEventDestroy(c->done);
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->staging) (void)hipFree(c->staging);
    if (c->mask) (void)hipFree(c->mask);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->pinned) (void)hipHostFree(c->pinned);
    if (c->queue) (void)hipFree(c->queue);
    if (c->tags) (void)hipFree(c->tags);
    delete c;
}

// Take a context from the scene's pool (a new one when all are in use).  The caller must hand it
// back with ctx_release; work it enqueued may still run (its `done` event orders the next user).
// `want`: the stream the caller will enqueue on (vr_render_tile_device), or none (the host-buffer
// entry points, which use the context's own stream).
int ctx_acquire(vr_scene* s, CallCtx** out, const hipStream_t* want = nullptr) {
    {
        // In order of preference:
        //  1. a free context whose last call's work has finished on the device (its `done` has
        //     completed);
        //  2. a free context whose last call was enqueued on the caller's own stream: stream order
        //     already puts the new call after that work, so the hipStreamWaitEvent on `done` costs
        //     nothing (bench.py's frames queue back to back on one stream and reuse ONE context --
        //     a second one would allocate a second frame-sized staging buffer, 68.7 GB at C4 / C5,
        //     inside the timed region, and its smaller cap could split alternate frames into passes);
        //  3. with none of those and fewer than two contexts, a new one (frame k + 1 on another
        //     stream then renders while frame k's launch drains); beyond two the most recent one is
        //     reused (its `done` orders the new call after it).
        std::lock_guard<std::mutex> g(s->ctx_mutex);
        for (size_t i = s->ctx_free.size(); i-- > 0;) {
            if (hipEventQuery(s->ctx_free[i]->done) == hipSuccess) {
                *out = s->ctx_free[i];
                s->ctx_free.erase(s->ctx_free.begin() + (ptrdiff_t)i);
                return VR_OK;
            }
        }
        if (want) {
            for (size_t i = s->ctx_free.size(); i-- > 0;) {
                if (s->ctx_free[i]->used && s->ctx_free[i]->last_stream == *want) {
                    *out = s->ctx_free[i];
                    s->ctx_free.erase(s->ctx_free.begin() + (ptrdiff_t)i);
                    return VR_OK;
                }
            }
        }
        if (!s->ctx_free.empty() && s->ctx_all.size() >= 2) {
            *out = s->ctx_free.back();
            s->ctx_free.pop_back();
            return VR_OK;
        }
    }
    CallCtx* c = new (std::nothrow) CallCtx();
    if (!c) return fail(VR_ERROR_OUT_OF_MEMORY, "call context allocation failed");
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    // blocking sync: a host-buffer call waits on `done` asleep, not spinning a core (8 spinning
    // callers under a 16-CPU quota throttled the whole process for ~10 ms at a time)
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->done, hipEventDisableTiming | hipEventBlockingSync);
#ifdef VR_COOP_PROF  // analysis builds: per-wave records after word 24 (vr_render.hip)
    if (e == hipSuccess) e = hipMalloc(&c->queue, 65536);
    if (e == hipSuccess) e = hipMemsetAsync(c->queue, 0, 65536, c->stream);
#else
    if (e == hipSuccess) e = hipMalloc(&c->queue, 256);
    if (e == hipSuccess) e = hipMemsetAsync(c->queue, 0, 256, c->stream);
#endif
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
        ctx_free_all(c);
        return fail(VR_ERROR_DEVICE, std::string("call context: ") + hipGetErrorString(e));
    }
    c->error = (int32_t*)(c->queue + 1);
    std::lock_guard<std::mutex> g(s->ctx_mutex);
    s->ctx_all.push_back(c);
    *out = c;
    return VR_OK;
}

void ctx_release(vr_scene* s, CallCtx* c) {
    std::lock_guard<std::mutex> g(s->ctx_mutex);
    s->ctx_free.push_back(c);
}

struct CtxLease {  // RAII hand-back
    vr_scene* s;
    CallCtx* c = nullptr;
    explicit CtxLease(vr_scene* sc) : s(sc) {}
    ~CtxLease() {
        if (c) ctx_release(s, c);
    }
};

// The sticky error word of `stream` (created zeroed on first use, on that stream).
int stream_slot(vr_scene* s, void* stream, int32_t** out) {
    std::lock_guard<std::mutex> g(s->slot_mutex);
    auto it = s->stream_slots.find(stream);
    if (it != s->stream_slots.end()) {
        *out = it->second;
        return VR_OK;
    }
    int32_t* p = nullptr;
    VR_HIP(hipMalloc(&p, 256));
    const hipError_t e = hipMemsetAsync(p, 0, 256, (hipStream_t)stream);
    if (e != hipSuccess) {
        (void)hipFree(p);
        return fail(VR_ERROR_DEVICE, std::string("error slot: ") + hipGetErrorString(e));
    }
    s->stream_slots.emplace(stream, p);
    *out = p;
    return VR_OK;
}

}  // namespace

extern "C" {

uint32_t vr_abi_version(void) { return VR_ABI_VERSION; }

const char* vr_last_error(void) { return g_last_error.c_str(); }

int vr_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int vr_spectrum_reflection_from_linear_rgb(double red, double green, double blue, double out[32]) {
    if (!out) return fail(VR_ERROR_INVALID_ARGUMENT, "null output");
    const double r = red, g = green, b = blue;
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
    for (int i = 0; i < 32; ++i)
        out[i] = c0 * vr_rgbspec_basis[VR_RGBSPEC_WHITE][i] + c1 * vr_rgbspec_basis[kx][i] +
                 c2 * vr_rgbspec_basis[ky][i];
    return VR_OK;
}

double vr_spectrum_intensity_at_wavelength(const vr_spectrum* sp, double wl) {
    if (!sp || sp->sample_count < 1) return 0.0;
    if (wl < sp->shortest_wavelength || wl > sp->longest_wavelength) return 0.0;
    const int n = (int)sp->sample_count;
    const double range = sp->longest_wavelength - sp->shortest_wavelength;
    const size_t i = (size_t)((double)(n - 1) * ((wl - sp->shortest_wavelength) / range));
    const double before = (double)i / (double)(n - 1) * range + sp->shortest_wavelength;
    if (i == (size_t)(n - 1)) return sp->samples[i];
    const double after = (double)(i + 1) / (double)(n - 1) * range + sp->shortest_wavelength;
    const double delta = after - before;
    const double ratio = (wl - before) / delta;
    return sp->samples[i] * (1.0 - ratio) + sp->samples[i + 1] * ratio;
}

static double gaussian_h(double wl, double alpha, double mu, double s1, double s2) {
    double s = wl < mu ? s1 : s2;
    double denominator = 2.0 * (s * s);
    double t = wl - mu;
    return alpha * std::exp(-(t * t) / denominator);
}

void vr_colour_xyz_for_wavelength(double wl, double out[3]) {
    out[0] = gaussian_h(wl, 1.056, 599.8, 37.9, 31.0) + gaussian_h(wl, 0.362, 442.0, 16.0, 26.7) +
             gaussian_h(wl, -0.065, 501.1, 20.4, 26.2);
    out[1] = gaussian_h(wl, 0.821, 568.8, 46.9, 40.5) + gaussian_h(wl, 0.286, 530.9, 16.3, 31.1);
    out[2] = gaussian_h(wl, 1.217, 437.0, 11.8, 36.0) + gaussian_h(wl, 0.681, 459.0, 26.0, 13.8);
}

int vr_scene_create(const vr_scene_desc* desc, int32_t device, uint32_t flags, vr_scene** out) {
    if (!desc || !out) return fail(VR_ERROR_INVALID_ARGUMENT, "null desc or out");
    *out = nullptr;
    vr_scene* s = new (std::nothrow) vr_scene();
    if (!s) return fail(VR_ERROR_OUT_OF_MEMORY, "scene allocation failed");
    s->device = device;
    s->host_only = (flags & VR_SCENE_HOST_ONLY) != 0;
    s->greedy_collapse = (flags & VR_SCENE_GREEDY_COLLAPSE) != 0;
    s->force_big = (flags & VR_SCENE_WIDE_OFFSETS) != 0;
    s->camera[0] = desc->camera_location.x;
    s->camera[1] = desc->camera_location.y;
    s->camera[2] = desc->camera_location.z;
    double extent = std::max({std::fabs(s->camera[0]), std::fabs(s->camera[1]), std::fabs(s->camera[2])});
    auto bad = [&](const std::string& m) {
        delete s;
        return fail(VR_ERROR_INVALID_ARGUMENT, m);
    };

    for (uint32_t i = 0; i < desc->material_count; ++i) {
        const vr_material_desc& m = desc->materials[i];
        if (m.kind < VR_MATERIAL_LAMBERTIAN || m.kind > VR_MATERIAL_DIELECTRIC) return bad("unknown material kind");
        if (m.colour.sample_count < 1 || m.colour.sample_count > VR_MAX_SPECTRUM_SAMPLES || !m.colour.samples)
            return bad("material spectrum needs 1..64 samples");
        vr::Material dm{};
        dm.kind = m.kind;
        dm.n = (int32_t)m.colour.sample_count;
        dm.shortest = m.colour.shortest_wavelength;
        dm.longest = m.colour.longest_wavelength;
        dm.diffuse = m.diffuse_strength;
        dm.reflection = m.reflection_strength;
        dm.smoothness = m.smoothness;
        std::memcpy(dm.samples, m.colour.samples, sizeof(double) * m.colour.sample_count);
        fill_knots(dm);
        s->materials.push_back(dm);
        if (vr_spectrum_intensity_at_wavelength(&m.colour, 0.0) != 0.0) s->dark0 = false;
        s->mats |= m.kind == VR_MATERIAL_LAMBERTIAN ? 1 : (m.kind == VR_MATERIAL_REFLECTIVE ? 2 : 4);
        // the dielectric's strength at 0 nm is not its eta(0): a path cut at the recursion limit
        // (lambda 0) needs the general lambda-0 chain
        if (m.kind == VR_MATERIAL_DIELECTRIC) s->dark0 = false;
    }
    // integrator: Whitted's ambient and light spectra become extra material rows
    if (desc->integrator && desc->integrator->kind == VR_INTEGRATOR_WHITTED) {
        const vr_integrator_desc& ig = *desc->integrator;
        if (ig.light_count > VR_MAX_LIGHTS || (ig.light_count && !ig.lights)) return bad("bad light list");
        auto spectrum_row = [&](const vr_spectrum& sp, vr::Material& dm) {
            if (sp.sample_count < 1 || sp.sample_count > VR_MAX_SPECTRUM_SAMPLES || !sp.samples) return false;
            dm = vr::Material{};
            dm.n = (int32_t)sp.sample_count;
            dm.shortest = sp.shortest_wavelength;
            dm.longest = sp.longest_wavelength;
            std::memcpy(dm.samples, sp.samples, sizeof(double) * sp.sample_count);
            fill_knots(dm);
            return true;
        };
        s->dev.integrator = VR_INTEGRATOR_WHITTED;
        s->dev.light_base = (int32_t)s->materials.size();
        s->dev.light_count = (int32_t)ig.light_count;
        vr::Material dm;
        if (!spectrum_row(ig.ambient_light, dm)) return bad("ambient light spectrum needs 1..64 samples");
        s->materials.push_back(dm);
        for (uint32_t j = 0; j < ig.light_count; ++j) {
            if (!spectrum_row(ig.lights[j].spectrum, dm)) return bad("light spectrum needs 1..64 samples");
            s->materials.push_back(dm);
            const vr_vec3& d = ig.lights[j].direction;
            s->light_dirs.insert(s->light_dirs.end(), {d.x, d.y, d.z});
        }
    } else if (desc->integrator && desc->integrator->kind != VR_INTEGRATOR_SIMPLE_RANDOM) {
        return bad("unknown integrator kind");
    }
    {  // the sky's lookup row (test_lighting_environment's RGB-basis spectrum: 32 samples)
        vr::Material sky{};
        sky.n = 32;
        sky.shortest = VR_RGBSPEC_SHORTEST;
        sky.longest = VR_RGBSPEC_LONGEST;
        fill_knots(sky);
        s->dev.sky_row = (int32_t)s->materials.size();
        s->materials.push_back(sky);
    }
    // objects: primitive lists keep their order; BVHs are built per mesh
    std::vector<int> mesh_object(desc->mesh_count, -1);
    for (uint32_t oi = 0; oi < desc->object_count; ++oi) {
        const vr_object_desc& o = desc->objects[oi];
        if (o.kind == VR_OBJECT_PRIMITIVE_LIST) {
            if ((uint64_t)o.first + o.count > desc->primitive_count) return bad("primitive list out of range");
            for (uint32_t k = 0; k < o.count; ++k) {
                const vr_primitive_desc& p = desc->primitives[o.first + k];
                if (p.material >= desc->material_count) return bad("primitive material out of range");
                vr::Prim dp{};
                dp.kind = p.kind;
                dp.material = (int32_t)p.material;
                dp.object = (int32_t)oi;
                dp.position = (int32_t)k;
                dp.scalar = p.scalar;
                if (p.kind == VR_PRIMITIVE_PLANE) {
                    // Plane::new (plane.rs:18-31)
                    H3 n = hnormalize({p.vector.x, p.vector.y, p.vector.z});
                    double ax = std::fabs(n.x), ay = std::fabs(n.y), az = std::fabs(n.z);
                    int k2 = ax < ay ? (ax < az ? 0 : 2) : (ay < az ? 1 : 2);  // smallest_coord
                    H3 axis{k2 == 0 ? 1.0 : 0.0, k2 == 1 ? 1.0 : 0.0, k2 == 2 ? 1.0 : 0.0};
                    H3 cot = hnormalize(hcross(n, axis));
                    H3 tan = hcross(n, cot);
                    dp.vec[0] = n.x; dp.vec[1] = n.y; dp.vec[2] = n.z;
                    dp.tan[0] = tan.x; dp.tan[1] = tan.y; dp.tan[2] = tan.z;
                    dp.cot[0] = cot.x; dp.cot[1] = cot.y; dp.cot[2] = cot.z;
                    dp.pre[0] = n.x * p.scalar; dp.pre[1] = n.y * p.scalar; dp.pre[2] = n.z * p.scalar;
                    extent = std::max(extent, std::fabs(p.scalar));
                } else if (p.kind == VR_PRIMITIVE_SPHERE) {
                    dp.vec[0] = p.vector.x; dp.vec[1] = p.vector.y; dp.vec[2] = p.vector.z;
                    dp.pre[0] = p.vector.x * p.vector.x;
                    dp.pre[1] = p.vector.y * p.vector.y;
                    dp.pre[2] = p.vector.z * p.vector.z;
                    dp.scalar2 = p.scalar * p.scalar;
                    extent = std::max({extent, std::fabs(p.vector.x) + std::fabs(p.scalar),
                                       std::fabs(p.vector.y) + std::fabs(p.scalar),
                                       std::fabs(p.vector.z) + std::fabs(p.scalar)});
                } else {
                    return bad("unknown primitive kind");
                }
                s->prims.push_back(dp);
            }
        } else if (o.kind == VR_OBJECT_BVH) {
            if (o.first >= desc->mesh_count) return bad("BVH object mesh out of range");
            if (mesh_object[o.first] >= 0) return bad("a mesh can back only one BVH object");
            mesh_object[o.first] = (int)oi;
        } else {
            return bad("unknown object kind");
        }
    }
    s->object_count = desc->object_count;
    // NaN-capable continuations (shading_finite): no early stop, the general lambda-0 chain
    if (s->mats & 4) s->nan_free = false;
    for (uint32_t mi = 0; mi < desc->mesh_count && s->nan_free; ++mi) {
        const vr_mesh_desc& m = desc->meshes[mi];
        if (mesh_object[mi] >= 0 && m.triangle_count && m.vertices && m.normals && !shading_finite(m))
            s->nan_free = false;
    }
    if (!s->nan_free) s->dark0 = false;
    s->leaf_order.resize(desc->mesh_count);
    s->mesh_tri_base.assign(desc->mesh_count, 0);
    // device build: requested, a device exists for it, and no NaN coordinate (the reference's
    // sort comparator maps NaN to Equal, which only the host build reproduces)
    s->device_bvh = (flags & (VR_SCENE_DEVICE_BVH | VR_SCENE_DEVICE_SAH)) != 0 && !s->host_only;
    s->device_sah = (flags & VR_SCENE_DEVICE_SAH) != 0 && (flags & VR_SCENE_REFERENCE_BVH) == 0;
    // traversal tree: SAH (default) or the reference's own median-split tree
    const bool sah = (flags & VR_SCENE_REFERENCE_BVH) == 0 && !s->device_bvh;
    for (uint32_t mi = 0; s->device_bvh && mi < desc->mesh_count; ++mi) {
        const vr_mesh_desc& m = desc->meshes[mi];
        if (m.triangle_count && !m.vertices) break;
        for (uint64_t i = 0; i < 9 * m.triangle_count; ++i)
            if (m.vertices[i] != m.vertices[i]) {
                s->device_bvh = false;
                break;
            }
    }
    for (uint32_t mi = 0; mi < desc->mesh_count; ++mi) {
        const vr_mesh_desc& m = desc->meshes[mi];
        if (m.triangle_count && (!m.vertices || !m.normals)) return bad("mesh without vertex or normal arrays");
        if (m.material >= desc->material_count) return bad("mesh material out of range");
        if (s->tri_count + m.triangle_count > (uint64_t)INT32_MAX) return bad("too many triangles (2^31)");
        if (s->device_bvh) {
            // shape and root box on the host (O(n)); the sort-based build runs after upload
            vr::Bvh bvh{};
            bvh.object = mesh_object[mi];
            bvh.tri_base = (int32_t)s->tri_count;
            bvh.material = (int32_t)m.material;
            s->mesh_tri_base[mi] = bvh.tri_base;
            Box3 rb = box_empty();
            for (uint64_t t = 0; t < m.triangle_count; ++t) {
                Box3 bb = box_empty();
                for (int k = 0; k < 3; ++k)
                    for (int c = 0; c < 3; ++c) {
                        const double v = m.vertices[9 * t + 3 * k + c];
                        bb.b[c] = iv_expand(bb.b[c], v);
                        extent = std::max(extent, std::fabs(v));
                    }
                rb = box_union(rb, bb);
            }
            if (m.triangle_count == 0) {
                bvh.root = INT32_MIN;
                for (int i = 0; i < 6; ++i) bvh.root_box[i] = (i & 1) ? -INFINITY : INFINITY;
            } else {
                box_to_layout(rb, bvh.root_box);
                bvh.root = m.triangle_count > 1 ? (int32_t)s->node_count : ~bvh.tri_base;
                s->pending.push_back({m.vertices, m.normals, m.triangle_count, (int32_t)s->node_count, bvh.tri_base, mi});
                s->max_depth = std::max(s->max_depth, 1);
            }
            s->leaf_order[mi].assign(m.triangle_count, 0);
            s->node_count += m.triangle_count ? m.triangle_count - 1 : 0;
            s->tri_count += m.triangle_count;
            if (mesh_object[mi] >= 0) s->bvhs.push_back(bvh);
            continue;
        }
        BvhBuilder B;
        std::vector<uint64_t> traversal_rank(m.triangle_count);
        B.tri_base = (int)s->tris.size();
        s->mesh_tri_base[mi] = B.tri_base;
        B.prims.resize(m.triangle_count);
        for (uint64_t t = 0; t < m.triangle_count; ++t) {
            Box3 bb = box_empty();  // BoundingBox::from_points(&vertices) (triangle.rs:101-105)
            for (int k = 0; k < 3; ++k)
                for (int c = 0; c < 3; ++c) {
                    double v = m.vertices[9 * t + 3 * k + c];
                    bb.b[c] = iv_expand(bb.b[c], v);
                    extent = std::max(extent, std::fabs(v));
                }
            B.prims[t].box = bb;
            for (int c = 0; c < 3; ++c) B.prims[t].centre[c] = (bb.b[c].min + bb.b[c].max) / 2.0;  // centre()
            B.prims[t].orig = t;
        }
        vr::Bvh bvh{};
        bvh.object = mesh_object[mi];
        bvh.tri_base = B.tri_base;
        bvh.material = (int32_t)m.material;
        if (m.triangle_count == 0) {
            bvh.root = INT32_MIN;
            for (int i = 0; i < 6; ++i) bvh.root_box[i] = (i & 1) ? -INFINITY : INFINITY;
        } else {
            Box3 rb;
            B.nodes.reserve(m.triangle_count);
            int32_t root = B.build(0, m.triangle_count, 0, rb);
            box_to_layout(rb, bvh.root_box);
            if (sah) {
                // the traversal tree: SAH over the reference-ordered triangles (orig = rank)
                std::vector<BuildPrim> sp(B.prims);
                for (uint64_t i = 0; i < m.triangle_count; ++i) sp[i].orig = i;
                SahBuilder T(sp);
                T.tri_base = B.tri_base;
                T.nodes.reserve(m.triangle_count);
                Box3 trb;
                root = T.build(0, m.triangle_count, 0, trb);
                B.nodes.swap(T.nodes);
                B.max_depth = T.max_depth;
                for (uint64_t i = 0; i < m.triangle_count; ++i) traversal_rank[i] = sp[i].orig;
            } else {
                for (uint64_t i = 0; i < m.triangle_count; ++i) traversal_rank[i] = i;
            }
            // re-base interior node indices into the scene-wide node array
            const int32_t node_base = (int32_t)s->nodes.size();
            for (auto& n : B.nodes)
                for (int c = 0; c < 2; ++c)
                    if (n.child[c] >= 0) n.child[c] += node_base;
            bvh.root = root >= 0 ? root + node_base : root;
            s->nodes.insert(s->nodes.end(), B.nodes.begin(), B.nodes.end());
            s->max_depth = std::max(s->max_depth, B.max_depth);
        }
        s->leaf_order[mi].resize(m.triangle_count);
        for (uint64_t i = 0; i < m.triangle_count; ++i) s->leaf_order[mi][i] = B.prims[i].orig;
        for (uint64_t i = 0; i < m.triangle_count; ++i) {
            const uint64_t r = traversal_rank[i];  // reference leaf position of traversal leaf i
            const uint64_t t = B.prims[r].orig;
            vr::TriVerts tv{};
            vr::TriNormals tn{};
            std::memcpy(tv.v, m.vertices + 9 * t, 9 * sizeof(double));
            std::memcpy(tn.n, m.normals + 9 * t, 9 * sizeof(double));
            tv.rank = (int64_t)B.tri_base + (int64_t)r;
            s->tris.push_back(tv);
            s->normals.push_back(tn);
        }
        if (mesh_object[mi] >= 0) s->bvhs.push_back(bvh);
        s->node_count = s->nodes.size();
        s->tri_count = s->tris.size();
    }
    // outward-rounded f32 root boxes (the kernel's pre-test)
    for (auto& b : s->bvhs)
        for (int k = 0; k < 6; ++k) b.root_box32[k] = (k % 2 == 0) ? round_lower(b.root_box[k]) : round_upper(b.root_box[k]);
    // BVH objects in object order (ties across objects depend on it)
    std::sort(s->bvhs.begin(), s->bvhs.end(), [](const vr::Bvh& a, const vr::Bvh& b) { return a.object < b.object; });
    // the render kernel's 4-wide tree (device builds: after the build, in upload)
    if (!s->device_bvh) collapse_wide(s, s->nodes);
    s->extent = extent;
    vr::DeviceScene& d = s->dev;
    d.prim_count = (int32_t)s->prims.size();
    d.bvh_count = (int32_t)s->bvhs.size();
    std::memcpy(d.camera, s->camera, sizeof d.camera);
    d.margin = 1e-9 * (extent + 1.0);
    d.behind_margin = 1e-6 * (extent + 1.0);
    d.extent = extent;
    if (!s->host_only) {
        int rc = upload(s);
        if (rc != VR_OK) {
            std::string msg = g_last_error;
            vr_scene_destroy(s);
            return fail(rc, msg);
        }
    }
    *out = s;
    return VR_OK;
}

void vr_scene_destroy(vr_scene* s) {
    if (!s) return;
    if (s->d_block || !s->ctx_all.empty() || !s->stream_slots.empty()) {
        (void)hipSetDevice(s->device);
        for (CallCtx* c : s->ctx_all) ctx_free_all(c);  // waits for each context's last work
        // (the streams may be gone by now: hipFree waits for the device instead)
        for (auto& kv : s->stream_slots) (void)hipFree(kv.second);
        if (s->d_block) (void)hipFree(s->d_block);
    }
    for (auto& kv : s->deferred)
        for (hipEvent_t e : kv.second.ev) (void)hipEventDestroy(e);
    delete s;
}

int vr_scene_get_info(const vr_scene* s, vr_scene_info* out) {
    if (!s || !out) return fail(VR_ERROR_INVALID_ARGUMENT, "null argument");
    out->triangle_count = s->tri_count;
    out->node_count = s->node_count;
    out->max_bvh_depth = (uint32_t)s->max_depth;
    out->object_count = s->object_count;
    out->extent = s->extent;
    out->device_bytes = s->device_bytes;
    out->wide_node_count = s->wide_count;
    out->traversal_stack = (uint32_t)s->wide_stack;
    out->flags = s->nan_free ? VR_SCENE_INFO_NAN_FREE : 0u;
    return VR_OK;
}

int vr_scene_set_staging_limit(vr_scene* s, uint64_t bytes) {
    if (!s) return fail(VR_ERROR_INVALID_ARGUMENT, "null scene");
    s->staging_limit = bytes;
    return VR_OK;
}

int vr_debug_set_fault_object(vr_scene* s, int32_t object) {
    if (!s) return fail(VR_ERROR_INVALID_ARGUMENT, "null scene");
    s->fault_object = object < 0 ? -1 : object;
    return VR_OK;
}

int vr_debug_set_launch_flags(vr_scene* s, uint32_t flags) {
    if (!s) return fail(VR_ERROR_INVALID_ARGUMENT, "null scene");
    const uint32_t allowed =
        VR_LAUNCH_NO_CULL | VR_LAUNCH_NO_DIST_CULL | VR_LAUNCH_NO_COOP | VR_LAUNCH_NO_LONE_WALK | VR_LAUNCH_STACK32;
    if (flags & ~allowed)
        return fail(VR_ERROR_INVALID_ARGUMENT,
                    "only NO_CULL / NO_DIST_CULL / NO_COOP / NO_LONE_WALK / STACK32 apply to every call");
    s->debug_launch_flags = flags;
    return VR_OK;
}

int vr_scene_needs_wide_offsets(uint64_t triangle_count, uint64_t wide_node_count) {
    return needs_big_offsets(triangle_count, wide_node_count) ? 1 : 0;
}

int vr_scene_bvh_nodes(const vr_scene* s, void* out) {
    if (!s || !out) return fail(VR_ERROR_INVALID_ARGUMENT, "null argument");
    const size_t bytes = s->node_count * sizeof(vr::Node);
    if (bytes == 0) return VR_OK;
    if (!s->device_bvh) {
        std::memcpy(out, s->nodes.data(), bytes);
        return VR_OK;
    }
    VR_HIP(hipSetDevice(s->device));
    VR_HIP(hipMemcpy(out, s->dev.nodes, bytes, hipMemcpyDeviceToHost));
    return VR_OK;
}

int vr_scene_bvh_leaf_order(const vr_scene* s, uint32_t mesh, uint64_t* out) {
    if (!s || !out || mesh >= s->leaf_order.size()) return fail(VR_ERROR_INVALID_ARGUMENT, "bad mesh index");
    std::memcpy(out, s->leaf_order[mesh].data(), sizeof(uint64_t) * s->leaf_order[mesh].size());
    return VR_OK;
}

namespace {
// Enqueue the render of params `p` into `state` on stream `st`, in passes that fit the context's
// staging buffer (16 B per pixel-sample: the final photon).  `err` is the device word the kernel
// flags a singular shading basis in.  Per-pass events of a timed launch: render kernel
// [start, mid), ordered reduce [mid, end).
struct PassEvents {
    std::vector<hipEvent_t> ev;
    ~PassEvents() {
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    }
    hipEvent_t add() {
        hipEvent_t e = nullptr;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        ev.push_back(e);
        return e;
    }
};

// Records the context's `done` on the call's stream when it goes out of scope, so that EVERY exit of
// a call after its first enqueue -- an error return included -- orders the context's next user
// (possibly on another stream) after the work this call left queued on its staging, mask, queue
// counter and scratch.  (The success paths record `done` themselves as well: recording it again
// at the same point of the stream changes nothing.)
struct DoneOnExit {
    hipEvent_t done;
    hipStream_t st;
    ~DoneOnExit() { (void)hipEventRecord(done, st); }
};


int enqueue_passes(vr_scene* s, CallCtx* c, const vr_render_params* p, double* state, hipStream_t st, int32_t* err,
                   bool counting, bool recording, void* records, unsigned long long* counters,
                   unsigned long long* wg_times, PassEvents* timing = nullptr, uint32_t launch_flags = 0,
                   uint32_t* variant = nullptr) {
    launch_flags |= s->debug_launch_flags;
    const bool no_cull = (launch_flags & VR_LAUNCH_NO_CULL) != 0;
    const uint64_t tw = p->tile.end_column - p->tile.start_column, th = p->tile.end_row - p->tile.start_row;
    const uint64_t npix = tw * th;
    if (npix == 0 || p->spp == 0) return VR_OK;
    size_t free_b = 0, total_b = 0;
    VR_HIP(hipMemGetInfo(&free_b, &total_b));
    // staging for a whole frame when half the free HBM holds it (a 288 GB MI355X: C4 / C5's
    // 68.7 GB on one GPU in one launch -- every extra launch adds the tail of the frame's longest
    // paths, ~7 ms on the C5 mesh); vr_scene_set_staging_limit lowers the cap (a GPU shared with
    // other work; the tests of the pass split)
    size_t cap = (free_b + c->staging_bytes) / 2;
    if (s->staging_limit) cap = std::min<size_t>(cap, s->staging_limit);
    uint64_t pass = recording ? p->spp : std::min<uint64_t>(p->spp, std::max<uint64_t>(1, cap / (16 * npix)));
    // the kernel decodes work items with 32-bit block indices: (8x8 blocks) x samples < 2^32
    if (((tw + 7) / 8) * ((th + 7) / 8) * pass >= (1ull << 32))
        return fail(VR_ERROR_UNSUPPORTED, "too many pixel blocks x samples in one launch (2^32)");
    // the context's previous user (possibly on another stream) must be done with its buffers
    VR_HIP(hipStreamWaitEvent(st, c->done, 0));
    DoneOnExit guard{c->done, st};
    c->last_stream = st;
    c->used = true;
    int rc = ctx_grow(&c->staging, &c->staging_bytes, (size_t)(16 * npix * pass), c->done);
    if (rc) return rc;
#ifdef VR_STAGE_GUARD
    if (c->tag_bytes < (size_t)(4 * npix * pass)) {
        rc = ctx_grow(&c->tags, &c->tag_bytes, (size_t)(4 * npix * pass), c->done);
        if (rc) return rc;
        VR_HIP(hipMemsetAsync(c->tags, 0, c->tag_bytes, st));  // generation 0: never written
    }
#endif
    // blocks whose camera rays all miss every object (one small kernel per call; VR_LAUNCH_NO_CULL
    // turns the test off: the records are the same bit for bit, tests/test_gpu_cull.py)
    const bool cull = !no_cull;
    const uint8_t* mask = nullptr;
    const uint32_t *live = nullptr, *live_count = nullptr;
    if (cull && !recording) {  // (the record variant writes every sample's record)
        // mask: 1 B per block; then the live-block list (4 B per block) and its count (16-B aligned)
        const uint64_t nb = ((tw + 7) / 8) * ((th + 7) / 8);
        const size_t list_off = (nb + 15) & ~(uint64_t)15;
        rc = ctx_grow(&c->mask, &c->mask_bytes, (size_t)(list_off + 4 * nb + 16), c->done);
        if (rc) return rc;
        if (nb >= (1ull << 32)) return fail(VR_ERROR_UNSUPPORTED, "too many pixel blocks in one tile (2^32)");
        vr::RenderArgs a = make_args(s, p, state);
        int lc = vr::launch_block_cull(a, (uint8_t*)c->mask, st);
        uint32_t* lst = (uint32_t*)((char*)c->mask + list_off);
        const char* bm = tuning_env("VR_BLOCK_MORTON");  // tuning hook: live blocks in Z-order
        const bool morton = bm ? atoi(bm) != 0 : (s->mats & 2) == 0;  // with block-major items (make_args)
        if (!lc)
            lc = vr::launch_block_compact((const uint8_t*)c->mask, (uint32_t)((tw + 7) / 8), (uint32_t)((th + 7) / 8),
                                          morton, lst, lst + nb, st);
        if (lc) return fail(VR_ERROR_DEVICE, vr::device_error_string(lc));
        mask = (const uint8_t*)c->mask;
        live = lst;
        live_count = lst + nb;
    }
    for (uint64_t done = 0; done < p->spp; done += pass) {
        vr_render_params q = *p;
        q.spp = (uint32_t)std::min<uint64_t>(pass, p->spp - done);
        q.first_sample = p->first_sample + done;
        q.accumulate = (done > 0 || p->accumulate) ? 1u : 0u;
        vr::RenderArgs a = make_args(s, &q, state);
        a.staging = (double*)c->staging;
        if (launch_flags & VR_LAUNCH_NO_DIST_CULL) {
            // every box the line crosses is walked (culled() / cull_far / cull_behind never prune):
            // the records stay the same bit for bit (tests/test_gpu_launch_variants.py)
            a.scene.margin = INFINITY;
            a.scene.behind_margin = INFINITY;
        }
        if (launch_flags & VR_LAUNCH_NO_COOP) a.coop = 0;
        if (launch_flags & VR_LAUNCH_NO_LONE_WALK) a.lone_walk = 0;
#ifdef VR_STAGE_GUARD
        a.stage_tag = (uint32_t*)c->tags;
        if (++c->gen == 0) c->gen = 1;
        a.stage_gen = c->gen;
#endif
        a.queue = c->queue;
        a.error_flag = err;
        a.block_mask = mask;
        a.live_blocks = live;
        a.live_count = live_count;
        a.records = records;
        a.counters = counters;
        a.wg_times = done == 0 ? wg_times : nullptr;
#ifdef VR_COOP_PROF  // analysis builds: the previous launch's tail-wave sums (vr_render.hip)
        {
            static unsigned long long h[16 + 6000];
            VR_HIP(hipStreamSynchronize(st));
            VR_HIP(hipMemcpy(h, c->queue + 8, sizeof h, hipMemcpyDeviceToHost));
            if (h[7])
                fprintf(stderr, "vrcoop A %llu coop %llu leaf %llu rest %llu iters %llu leafrounds %llu phaseA %llu waves %llu maxwall %llu sumwall %llu lone %llu\n",
                        h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9], h[10]);
            for (unsigned long long i = 0; i < h[11] && i < 1000; ++i)
                fprintf(stderr, "vrwave %llu %llu %llu %llu %llu %llu\n", h[16 + 6 * i], h[17 + 6 * i], h[18 + 6 * i],
                        h[19 + 6 * i], h[20 + 6 * i], h[21 + 6 * i]);
            VR_HIP(hipMemset(c->queue + 8, 0, sizeof h));
        }
#endif
        VR_HIP(hipMemsetAsync(c->queue, 0, sizeof(unsigned long long), st));
        hipEvent_t mid = nullptr;
        if (timing) {
            hipEvent_t start = timing->add();
            mid = timing->add();
            if (!start || !mid) return fail(VR_ERROR_DEVICE, "hipEventCreate failed");
            VR_HIP(hipEventRecord(start, st));
        }
        // LDS stack entries: the 4-wide walk's, and the binary walk's for Whitted shadow rays
        const int stack = s->dev.integrator == 1 ? std::max(stack_depth(s), wide_stack_depth(s)) : wide_stack_depth(s);
        vr::LaunchChoice lc;
        lc.stack_depth = stack;
        lc.counting = counting;
        lc.recording = recording;
        lc.dark0 = s->dark0;
        lc.mats = s->mats ? s->mats : 3;
        lc.big = needs_big_offsets(s);
        // the cooperative tail's instantiations exist for DARK0 scenes with a reflective material
        lc.coop = a.coop != 0 && !recording && !counting && !lc.big && s->dev.integrator != 1 && s->dark0 &&
                  (lc.mats & 2);
        // 16-bit LDS stack entries: every node index of the tree fits (round 6, vr_render.hip
        // launch_render_t; VR_LAUNCH_STACK32 keeps 32-bit entries, the same records bit for bit)
        lc.s16 = !recording && !counting && !lc.big && !lc.coop && s->dev.integrator != 1 && s->wide_count < 65536 &&
                 stack <= 32 && !(launch_flags & VR_LAUNCH_STACK32);
        if (variant)
            *variant = (lc.coop ? VR_VARIANT_COOP : 0u) | (lc.big ? VR_VARIANT_WIDE_OFFSETS : 0u) |
                       (lc.s16 ? VR_VARIANT_STACK16 : 0u);
        // the COOP instantiations (2 waves per SIMD) keep 3 workgroups per CU (coop_grid_per_cu)
        const int per_cu = lc.coop ? coop_grid_per_cu() : grid_per_cu();
        int lr = vr::launch_render(a, lc, std::max(1, s->cu_count) * per_cu, st, mid);
        if (lr) return fail(lr == -1000 ? VR_ERROR_UNSUPPORTED : VR_ERROR_DEVICE, vr::device_error_string(lr));
        if (timing) {
            hipEvent_t end = timing->add();
            if (!end) return fail(VR_ERROR_DEVICE, "hipEventCreate failed");
            VR_HIP(hipEventRecord(end, st));
        }
    }
    VR_HIP(hipEventRecord(c->done, st));
    return VR_OK;
}

// Scratch of a host-buffer call: device records (64 B per pixel) then the host layout
// (88 B per pixel: colour, colour_sum, colour_bias, weight, weight_bias back to back).
int host_call_scratch(CallCtx* c, uint64_t npix, size_t extra, double** state, double** planar, void** rest) {
    const size_t rec = (npix * 64 + 255) & ~size_t(255), pl = (npix * 88 + 255) & ~size_t(255);
    int rc = ctx_grow(&c->scratch, &c->scratch_bytes, rec + pl + extra, c->done);
    if (rc) return rc;
    *state = (double*)c->scratch;
    if (planar) *planar = (double*)((char*)c->scratch + rec);
    if (rest) *rest = (char*)c->scratch + rec + pl;
    return VR_OK;
}
}  // namespace

int vr_render_tile_device(const vr_scene* s, const vr_render_params* p, double* state, void* stream,
                          uint32_t launch_flags, vr_launch_stats* stats) {
    int rc = check_render_params(s, p);
    if (rc) return rc;
    if (!state) return fail(VR_ERROR_INVALID_ARGUMENT, "null state");
    VR_HIP(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)stream;
    vr_scene* ms = const_cast<vr_scene*>(s);
    const bool counting = (launch_flags & VR_LAUNCH_COUNTERS) != 0;
    const bool timed = (launch_flags & VR_LAUNCH_TIMED) != 0 || counting;
    // timed without waiting: the events stay with the scene until vr_collect_launch_times
    const bool defer = timed && !counting && (launch_flags & VR_LAUNCH_DEFER_TIMES) != 0;
    int32_t* slot = nullptr;
    rc = stream_slot(ms, stream, &slot);
    if (rc) return rc;
    if (defer) {  // a caller that defers must collect: the pending events are bounded per stream
        std::lock_guard<std::mutex> g(ms->slot_mutex);
        auto it = ms->deferred.find(stream);
        if (it != ms->deferred.end() && it->second.passes.size() >= vr::kMaxDeferredLaunches)
            return fail(VR_ERROR_INVALID_ARGUMENT,
                        "too many VR_LAUNCH_DEFER_TIMES launches on this stream without vr_collect_launch_times");
    }
    std::unique_lock<std::mutex> lock(ms->counter_mutex, std::defer_lock);
    // diagnostic (tools): with counters, VR_WG_TIMES_PATH receives per-workgroup start/end stamps
    const char* wg_path = counting ? tuning_env("VR_WG_TIMES_PATH") : nullptr;
    CallScratch wg;
    const uint64_t blocks = (uint64_t)std::max(1, s->cu_count) * grid_per_cu();  // persistent grid limit
    unsigned long long* counters = nullptr;
    if (counting) {
        lock.lock();
        VR_HIP(hipMemsetAsync(s->d_counters, 0, sizeof(unsigned long long) * vr::kCntCount, st));
        counters = s->d_counters;
        if (wg_path) VR_HIP(hipMalloc(&wg.ptr, blocks * 2 * sizeof(unsigned long long)));
    }
    PassEvents pe;
    uint32_t variant = 0;
    {
        CtxLease L(ms);
        rc = ctx_acquire(ms, &L.c, &st);
        if (rc) return rc;
        rc = enqueue_passes(ms, L.c, p, state, st, slot, counting, false, nullptr, counters,
                            (unsigned long long*)wg.ptr, timed ? &pe : nullptr, launch_flags, &variant);
        if (rc) return rc;
    }
    if (!timed) {  // errors of this launch: vr_stream_check_error(scene, stream)
        if (stats) {
            std::memset(stats, 0, sizeof *stats);
            stats->variant = variant;
        }
        return VR_OK;
    }
    if (defer) {
        std::lock_guard<std::mutex> g(ms->slot_mutex);
        vr_scene::Deferred& d = ms->deferred[stream];
        d.ev.insert(d.ev.end(), pe.ev.begin(), pe.ev.end());
        d.passes.push_back((uint32_t)(pe.ev.size() / 3));
        pe.ev.clear();  // owned by the scene now
        if (stats) {
            std::memset(stats, 0, sizeof *stats);
            stats->passes = d.passes.back();
            stats->variant = variant;
        }
        return VR_OK;
    }
    float render_ms = 0.f, reduce_ms = 0.f;
    if (!pe.ev.empty()) VR_HIP(hipEventSynchronize(pe.ev.back()));
    for (size_t i = 0; i + 3 <= pe.ev.size(); i += 3) {
        float x = 0.f, y = 0.f;
        VR_HIP(hipEventElapsedTime(&x, pe.ev[i], pe.ev[i + 1]));
        VR_HIP(hipEventElapsedTime(&y, pe.ev[i + 1], pe.ev[i + 2]));
        render_ms += x;
        reduce_ms += y;
    }
    if (stats) {
        std::memset(stats, 0, sizeof *stats);
        stats->kernel_ms = render_ms;
        stats->reduce_ms = reduce_ms;
        stats->passes = (uint32_t)(pe.ev.size() / 3);
        stats->variant = variant;
        stats->timed = 1;
    }
    if (counting) {
        unsigned long long c[vr::kCntCount];
        VR_HIP(hipMemcpy(c, s->d_counters, sizeof c, hipMemcpyDeviceToHost));
        if (const char* cp = tuning_env("VR_COUNTERS_PATH")) {  // diagnostic: the raw counter array
            if (FILE* f = std::fopen(cp, "wb")) {
                std::fwrite(c, sizeof c, 1, f);
                std::fclose(f);
            }
        }
        if (wg_path && wg.ptr) {
            std::vector<unsigned long long> t(blocks * 2);
            VR_HIP(hipMemcpy(t.data(), wg.ptr, t.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
            if (FILE* f = std::fopen(wg_path, "wb")) {
                std::fwrite(t.data(), sizeof(unsigned long long), t.size(), f);
                std::fclose(f);
            }
        }
        if (stats) {
            stats->box_tests = c[vr::kCntBoxTests];
            stats->node_visits = c[vr::kCntNodeVisits];
            stats->triangle_tests = c[vr::kCntTriangleTests];
            stats->rays = c[vr::kCntRays];
            stats->shaded_triangle_hits = c[vr::kCntShadedTriangles];
            stats->samples = c[vr::kCntSamples];
            stats->traversal_slots = c[vr::kCntTraversalSlots];
            stats->path_loop_slots = c[vr::kCntOuterSlots];
            stats->exact_box_tests = c[vr::kCntExactBoxes];
        }
    }
    return read_and_clear_error(slot, st);
}

int vr_collect_launch_times(const vr_scene* s, void* stream, vr_launch_times* out) {
    if (!s || !out) return fail(VR_ERROR_INVALID_ARGUMENT, "null argument");
    if (s->host_only) return fail(VR_ERROR_HOST_ONLY, "scene was created with VR_SCENE_HOST_ONLY");
    VR_HIP(hipSetDevice(s->device));
    vr_scene* ms = const_cast<vr_scene*>(s);
    vr_scene::Deferred d;
    int32_t* slot = nullptr;
    {
        std::lock_guard<std::mutex> g(ms->slot_mutex);
        auto it = ms->deferred.find(stream);
        if (it != ms->deferred.end()) {
            d = std::move(it->second);
            ms->deferred.erase(it);
        }
        auto sl = ms->stream_slots.find(stream);
        if (sl != ms->stream_slots.end()) slot = sl->second;
    }
    PassEvents pe;  // destroys the events on every exit
    pe.ev = std::move(d.ev);
    std::memset(out, 0, sizeof *out);
    if (!pe.ev.empty()) VR_HIP(hipEventSynchronize(pe.ev.back()));
    for (size_t i = 0; i + 3 <= pe.ev.size(); i += 3) {
        float x = 0.f, y = 0.f;
        VR_HIP(hipEventElapsedTime(&x, pe.ev[i], pe.ev[i + 1]));
        VR_HIP(hipEventElapsedTime(&y, pe.ev[i + 1], pe.ev[i + 2]));
        out->kernel_ms += x;
        out->reduce_ms += y;
    }
    out->launches = (uint32_t)d.passes.size();
    for (uint32_t n : d.passes) {
        out->passes += n;
        out->max_passes = std::max(out->max_passes, n);
    }
    // the device errors of those launches, as a timed launch reports its own
    return slot ? read_and_clear_error(slot, (hipStream_t)stream) : VR_OK;
}

int vr_stream_check_error(const vr_scene* s, void* stream) {
    if (!s) return fail(VR_ERROR_INVALID_ARGUMENT, "null scene");
    if (s->host_only) return fail(VR_ERROR_HOST_ONLY, "scene was created with VR_SCENE_HOST_ONLY");
    VR_HIP(hipSetDevice(s->device));
    int32_t* slot = nullptr;
    {
        vr_scene* ms = const_cast<vr_scene*>(s);
        std::lock_guard<std::mutex> g(ms->slot_mutex);
        auto it = ms->stream_slots.find(stream);
        if (it != ms->stream_slots.end()) slot = it->second;
    }
    if (!slot) {  // nothing of this scene was ever launched on the stream
        VR_HIP(hipStreamSynchronize((hipStream_t)stream));
        return VR_OK;
    }
    return read_and_clear_error(slot, (hipStream_t)stream);
}

int vr_render_tile(const vr_scene* s, const vr_render_params* p, vr_accumulation_buffer* buf) {
    int rc = check_render_params(s, p);
    if (rc) return rc;
    const uint64_t tw = p->tile.end_column - p->tile.start_column, th = p->tile.end_row - p->tile.start_row;
    if (!buf || buf->width != tw || buf->height != th || !buf->colour || !buf->colour_sum || !buf->colour_bias ||
        !buf->weight || !buf->weight_bias)
        return fail(VR_ERROR_INVALID_ARGUMENT, "accumulation buffer does not match the tile");
    const uint64_t n = tw * th;
    if (n == 0) return VR_OK;
    VR_HIP(hipSetDevice(s->device));
    vr_scene* ms = const_cast<vr_scene*>(s);
    CtxLease L(ms);
    rc = ctx_acquire(ms, &L.c);
    if (rc) return rc;
    CallCtx* c = L.c;
    const hipStream_t st = c->stream;
    VR_HIP(hipStreamWaitEvent(st, c->done, 0));
    DoneOnExit guard{c->done, st};
    double *state = nullptr, *planar = nullptr;
    rc = host_call_scratch(c, n, 0, &state, &planar, nullptr);
    if (rc) return rc;
    // one sample into a fresh buffer (vr_partial_render_scene, the reference's per-call pattern):
    // only colour_sum comes back (24 B per pixel), the host derives the other four arrays
    const bool fresh1 = !p->accumulate && p->spp == 1;
    const size_t payload = (fresh1 ? 24 : 88) * n;
    rc = ctx_grow_pinned(c, payload + 256);  // + the call's error word
    if (rc) return rc;
    double* host = (double*)c->pinned;  // same layout as `planar`
    const size_t b3 = n * 3 * sizeof(double), b1 = n * sizeof(double);
    if (p->accumulate) {  // continue update_pixel from the caller's buffer
        parallel_copy(host + 3 * n, buf->colour_sum, b3);
        parallel_copy(host + 6 * n, buf->colour_bias, b3);
        parallel_copy(host + 9 * n, buf->weight, b1);
        parallel_copy(host + 10 * n, buf->weight_bias, b1);
        VR_HIP(hipMemcpyAsync(planar + 3 * n, host + 3 * n, 2 * b3 + 2 * b1, hipMemcpyHostToDevice, st));
        const int e = vr::launch_buffer_convert(planar, state, n, 0, st);
        if (e) return fail(VR_ERROR_DEVICE, std::string("buffer import: ") + hipGetErrorString((hipError_t)e));
    } else {  // AccumulationBuffer::new
        VR_HIP(hipMemsetAsync(state, 0, n * 64, st));
    }
    rc = enqueue_passes(ms, c, p, state, st, c->error, false, false, nullptr, nullptr, nullptr);
    if (rc) return rc;
    const int e = vr::launch_buffer_convert(state, planar, n, fresh1 ? 2 : 1, st);
    if (e) return fail(VR_ERROR_DEVICE, std::string("buffer export: ") + hipGetErrorString((hipError_t)e));
    VR_HIP(hipMemcpyAsync(host, planar, fresh1 ? b3 : 3 * b3 + 2 * b1, hipMemcpyDeviceToHost, st));
    volatile int32_t* flag = (volatile int32_t*)((char*)host + payload);  // the error word rides along
    VR_HIP(hipMemcpyAsync((void*)flag, c->error, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    VR_HIP(hipEventRecord(c->done, st));
    static const bool host_timing = tuning_env("VR_HOST_TIMING") != nullptr;  // diagnostic (tools/dropin.py)
    const auto t_enq = std::chrono::steady_clock::now();
    VR_HIP(hipEventSynchronize(c->done));
    if (*flag) {
        VR_HIP(hipMemsetAsync(c->error, 0, sizeof(int32_t), st));
        VR_HIP(hipStreamSynchronize(st));
        return fail(VR_ERROR_SINGULAR_BASIS,
                    "Normal, tangent and cotangent don't form a valid basis (det == 0); the reference panics here");
    }
    const auto t_dev = std::chrono::steady_clock::now();
    struct Report {
        bool on;
        std::chrono::steady_clock::time_point a, b;
        ~Report() {
            if (on)
                std::fprintf(stderr, "vr_render_tile host timing: device wait %.3f ms, host copy-out %.3f ms\n",
                             std::chrono::duration<double, std::milli>(b - a).count(),
                             std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - b).count());
        }
    } report{host_timing, t_enq, t_dev};
    if (fresh1) {
        // update_pixel (accumulation_buffer.rs:44-60) from zeros with weight 1: weight 1, weight bias
        // (1 - 0) - 1 = 0; colour_sum t = 0 + y with y = c * 1 - 0, so y == t bit for bit except y = -0
        // (t = +0), where the bias (t - 0) - y is +0 either way; colour = t * (1 / 1)
        parallel_range(n, (uint64_t)1 << 14, [&](uint64_t b, uint64_t e) {
            for (uint64_t i = b; i < e; ++i) {
                for (int k = 0; k < 3; ++k) {
                    const double t = host[3 * i + k];
                    buf->colour_sum[3 * i + k] = t;
                    buf->colour_bias[3 * i + k] = (t - 0.0) - t;
                    buf->colour[3 * i + k] = t * (1.0 / 1.0);
                }
                buf->weight[i] = 1.0;
                buf->weight_bias[i] = 0.0;
            }
        });
    } else {
        parallel_copy(buf->colour, host, b3);
        parallel_copy(buf->colour_sum, host + 3 * n, b3);
        parallel_copy(buf->colour_bias, host + 6 * n, b3);
        parallel_copy(buf->weight, host + 9 * n, b1);
        parallel_copy(buf->weight_bias, host + 10 * n, b1);
    }
    return VR_OK;
}

int vr_partial_render_scene(const vr_scene* s, vr_tile tile, uint64_t height, uint64_t width,
                            vr_accumulation_buffer* out) {
    if (!s) return fail(VR_ERROR_INVALID_ARGUMENT, "null scene");
    vr_render_params p{};
    p.tile = tile;
    p.height = height;
    p.width = width;
    p.spp = 1;
    p.accumulate = 0;
    p.seed = s->partial_seed;
    p.first_sample = const_cast<vr_scene*>(s)->pass_counter.fetch_add(1);
    return vr_render_tile(s, &p, out);
}

int vr_render_samples(const vr_scene* s, const vr_render_params* p, vr_sample_record* out) {
    int rc = check_render_params(s, p);
    if (rc) return rc;
    if (!out) return fail(VR_ERROR_INVALID_ARGUMENT, "null output");
    const uint64_t tw = p->tile.end_column - p->tile.start_column, th = p->tile.end_row - p->tile.start_row;
    const uint64_t n = tw * th;
    if (n == 0 || p->spp == 0) return VR_OK;
    VR_HIP(hipSetDevice(s->device));
    vr_scene* ms = const_cast<vr_scene*>(s);
    CtxLease L(ms);
    rc = ctx_acquire(ms, &L.c);
    if (rc) return rc;
    CallCtx* c = L.c;
    const hipStream_t st = c->stream;
    VR_HIP(hipStreamWaitEvent(st, c->done, 0));
    DoneOnExit guard{c->done, st};
    const size_t rec_bytes = n * p->spp * sizeof(vr_sample_record);
    double* state = nullptr;
    void* rec = nullptr;
    rc = host_call_scratch(c, n, rec_bytes, &state, nullptr, &rec);
    if (rc) return rc;
    VR_HIP(hipMemsetAsync(state, 0, n * 64, st));
    vr_render_params q = *p;
    q.accumulate = 0;
    rc = enqueue_passes(ms, c, &q, state, st, c->error, false, true, rec, nullptr, nullptr);
    if (rc) return rc;
    VR_HIP(hipMemcpyAsync(out, rec, rec_bytes, hipMemcpyDeviceToHost, st));
    VR_HIP(hipEventRecord(c->done, st));
    return read_and_clear_error(c->error, st);
}

int vr_trace_rays(const vr_scene* s, uint64_t n, const double* origins, const double* directions,
                  vr_hit_record* out) {
    if (!s || (n && (!origins || !directions || !out))) return fail(VR_ERROR_INVALID_ARGUMENT, "null argument");
    if (s->host_only) return fail(VR_ERROR_HOST_ONLY, "scene was created with VR_SCENE_HOST_ONLY");
    if (n == 0) return VR_OK;
    VR_HIP(hipSetDevice(s->device));
    vr_scene* ms = const_cast<vr_scene*>(s);
    CtxLease L(ms);
    int rc = ctx_acquire(ms, &L.c);
    if (rc) return rc;
    CallCtx* c = L.c;
    const hipStream_t st = c->stream;
    VR_HIP(hipStreamWaitEvent(st, c->done, 0));
    DoneOnExit guard{c->done, st};
    const size_t in_bytes = n * 3 * sizeof(double), out_bytes = n * sizeof(vr_hit_record);
    rc = ctx_grow(&c->scratch, &c->scratch_bytes, 2 * in_bytes + out_bytes, c->done);
    if (rc) return rc;
    char* b = (char*)c->scratch;
    VR_HIP(hipMemcpyAsync(b, origins, in_bytes, hipMemcpyHostToDevice, st));
    VR_HIP(hipMemcpyAsync(b + in_bytes, directions, in_bytes, hipMemcpyHostToDevice, st));
    VR_HIP(hipMemsetAsync(b + 2 * in_bytes, 0, out_bytes, st));
    vr::TraceArgs a{};
    a.scene = s->dev;
    a.n = n;
    a.origins = (const double*)b;
    a.directions = (const double*)(b + in_bytes);
    a.out = b + 2 * in_bytes;
    int lr = vr::launch_trace(a, stack_depth(s), st);
    if (lr) return fail(lr == -1000 ? VR_ERROR_UNSUPPORTED : VR_ERROR_DEVICE, vr::device_error_string(lr));
    VR_HIP(hipMemcpyAsync(out, b + 2 * in_bytes, out_bytes, hipMemcpyDeviceToHost, st));
    VR_HIP(hipEventRecord(c->done, st));
    VR_HIP(hipStreamSynchronize(st));
    return VR_OK;
}

int vr_merge_tile(vr_accumulation_buffer* dst, vr_tile t, const vr_accumulation_buffer* src) {
    if (!dst || !src || !dst->colour || !dst->weight || !src->colour || !src->weight)
        return fail(VR_ERROR_INVALID_ARGUMENT, "null buffer");
    // accumulation_buffer.rs:63-64 assert the tile size; Array2D indexing asserts the bounds
    if (t.end_column < t.start_column || t.end_row < t.start_row || t.end_column > dst->width ||
        t.end_row > dst->height || src->width != t.end_column - t.start_column ||
        src->height != t.end_row - t.start_row)
        return fail(VR_ERROR_INVALID_ARGUMENT, "merge_tile: tile does not match the buffers");
    // blend (accumulation_buffer.rs:87-91) per pixel; rows are independent, so a large tile is
    // split into row bands over host threads (96 B of memory traffic per pixel: one core merged
    // a 1024^2 frame in ~5 ms, the bottleneck of main.rs's one merging thread)
    auto rows = [&](uint64_t r0, uint64_t r1) {
        for (uint64_t i = r0; i < r1; ++i) {
            for (uint64_t j = 0; j < src->width; ++j) {
                const uint64_t d = (t.start_row + i) * dst->width + (t.start_column + j), q = i * src->width + j;
                const double w1 = dst->weight[d], w2 = src->weight[q];
                const double inv = 1.0 / (w1 + w2);
                for (int k = 0; k < 3; ++k)
                    dst->colour[3 * d + k] = (dst->colour[3 * d + k] * w1 + src->colour[3 * q + k] * w2) * inv;
                dst->weight[d] = w1 + w2;
            }
        }
    };
    parallel_range(src->height, std::max<uint64_t>(1, ((uint64_t)1 << 16) / std::max<uint64_t>(1, src->width)), rows);
    return VR_OK;
}

int vr_resolve_state(const double* state, uint64_t pixel_count, double* colour) {
    if (!state || !colour) return fail(VR_ERROR_INVALID_ARGUMENT, "null argument");
    for (uint64_t i = 0; i < pixel_count; ++i) {  // the sums half of the records (vr_layout.h)
        const double w = state[4 * i + 3];
        const double inv = 1.0 / w;
        for (int k = 0; k < 3; ++k) colour[3 * i + k] = w != 0.0 ? state[4 * i + k] * inv : 0.0;
    }
    return VR_OK;
}

// mesh::load_obj (src/mesh.rs:13-88) over the obj 0.9 crate's parsing: "v x y z" and
// "vn x y z" as f32 (correctly rounded strtof) widened to f64, "f a b c ..." with a, a/t,
// a//n or a/t/n corners (1-based, negative = relative), fan triangles (v0, v_i, v_{i+1}).
int vr_load_obj(const char* path, uint64_t* triangle_count, double** vertices, double** normals) {
    if (!path || !triangle_count || !vertices || !normals) return fail(VR_ERROR_INVALID_ARGUMENT, "null argument");
    FILE* f = std::fopen(path, "rb");
    if (!f) return fail(VR_ERROR_IO, std::string("cannot open ") + path);
    std::vector<float> pos, nrm;
    size_t tex_count = 0;
    struct Corner {
        int64_t v, n;
    };
    std::vector<double> vout, nout;
    std::vector<Corner> poly;
    char* line = nullptr;
    size_t cap = 0;
    int64_t lineno = 0;
    // obj 0.9: 1-based indices, negative = relative to the elements read so far, 0 invalid
    auto resolve = [](long long idx, size_t count) -> int64_t {
        if (idx > 0) return (int64_t)idx - 1;
        if (idx < 0) return (int64_t)count + idx;
        return -1;
    };
    auto is_space = [](char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\f' || c == '\v'; };
    // exactly `n` f32 fields (Rust's correctly rounded str::parse::<f32>, here strtof), then an
    // optional extra field (the w of "v x y z w") and the end of the line
    auto floats = [&](char* e, float* out, int n, int max_fields) -> bool {
        int got = 0;
        while (true) {
            while (*e && is_space(*e)) ++e;
            if (*e == '\0' || *e == '#') break;
            char* q;
            const float v = std::strtof(e, &q);
            if (q == e || (*q && !is_space(*q) && *q != '#')) return false;
            if (got < n) out[got] = v;
            ++got;
            e = q;
        }
        return got >= n && got <= max_fields;
    };
    int status = VR_OK;
    std::string err;
    while (getline(&line, &cap, f) != -1) {
        ++lineno;
        char* s = line;
        while (*s == ' ' || *s == '\t') ++s;
        if (s[0] == 'v' && is_space(s[1])) {
            float xyz[3];
            if (!floats(s + 1, xyz, 3, 4)) {
                status = VR_ERROR_IO;
                err = "malformed vertex at line " + std::to_string(lineno);
                break;
            }
            pos.insert(pos.end(), xyz, xyz + 3);
        } else if (s[0] == 'v' && s[1] == 'n' && is_space(s[2])) {
            float xyz[3];
            if (!floats(s + 2, xyz, 3, 3)) {
                status = VR_ERROR_IO;
                err = "malformed normal at line " + std::to_string(lineno);
                break;
            }
            nrm.insert(nrm.end(), xyz, xyz + 3);
        } else if (s[0] == 'v' && s[1] == 't' && is_space(s[2])) {
            ++tex_count;  // texture coordinates: only counted, for index validation (mesh.rs:19)
        } else if (s[0] == 'f' && is_space(s[1])) {
            poly.clear();
            char* e = s + 1;
            while (true) {
                while (*e && is_space(*e)) ++e;
                if (*e == '\0' || *e == '#') break;
                char* q;
                const long long vi = std::strtoll(e, &q, 10);
                bool ok = q != e;
                e = q;
                long long ti = 0, ni = 0;
                if (ok && *e == '/') {
                    ++e;
                    if (*e != '/') {
                        ti = std::strtoll(e, &q, 10);
                        ok = q != e;
                        e = q;
                    }
                    if (ok && *e == '/') {
                        ++e;
                        ni = std::strtoll(e, &q, 10);
                        ok = q != e;
                        e = q;
                    }
                }
                if (!ok || (*e && !is_space(*e) && *e != '#')) {
                    status = VR_ERROR_IO;
                    err = "malformed face at line " + std::to_string(lineno);
                    break;
                }
                const Corner c{resolve(vi, pos.size() / 3), ni ? resolve(ni, nrm.size() / 3) : -1};
                const int64_t t = ti ? resolve(ti, tex_count) : 0;
                if (c.v < 0 || (size_t)c.v >= pos.size() / 3 || (ni && (c.n < 0 || (size_t)c.n >= nrm.size() / 3)) ||
                    (ti && (t < 0 || (size_t)t >= tex_count))) {
                    status = VR_ERROR_IO;
                    err = "face index out of range at line " + std::to_string(lineno);
                    break;
                }
                poly.push_back(c);
            }
            if (status != VR_OK) break;
            // get_triangles (mesh.rs:43-72): fan (v0, v_i, v_{i+1}); fewer than 3 corners: none
            for (size_t i = 1; i + 1 < poly.size(); ++i) {
                const Corner cs3[3] = {poly[0], poly[i], poly[i + 1]};
                for (const Corner& c : cs3) {
                    for (int k = 0; k < 3; ++k) vout.push_back((double)pos[3 * c.v + k]);
                    for (int k = 0; k < 3; ++k) nout.push_back(c.n >= 0 ? (double)nrm[3 * c.n + k] : 0.0);
                }
            }
        }
        // everything else (comments, o, g, s, usemtl, mtllib, l, p, blank lines) carries no
        // geometry for load_obj: objects and groups are flattened in file order (mesh.rs:82-85)
    }
    std::free(line);
    std::fclose(f);
    if (status != VR_OK) return fail(status, err);
    const uint64_t n = vout.size() / 9;
    double* v = (double*)std::malloc(sizeof(double) * std::max<size_t>(vout.size(), 1));
    double* nn = (double*)std::malloc(sizeof(double) * std::max<size_t>(nout.size(), 1));
    if (!v || !nn) {
        std::free(v);
        std::free(nn);
        return fail(VR_ERROR_OUT_OF_MEMORY, "mesh allocation failed");
    }
    std::memcpy(v, vout.data(), sizeof(double) * vout.size());
    std::memcpy(nn, nout.data(), sizeof(double) * nout.size());
    *triangle_count = n;
    *vertices = v;
    *normals = nn;
    return VR_OK;
}

void vr_mesh_free(double* vertices, double* normals) {
    std::free(vertices);
    std::free(normals);
}

// ---------------------------------------------------------------------------------------------
// Display end: ClampingToneMapper over ColourXyz::to_srgb (image.rs:166-187,
// colour_xyz.rs:49-84) on the device, ImageRgbU8::write_png (image.rs:52-66) on the host.
// ---------------------------------------------------------------------------------------------
int vr_tone_map_device(const double* state, uint64_t pixel_count, uint8_t* rgb_out, int device, void* stream) {
    if (!state || !rgb_out) return fail(VR_ERROR_INVALID_ARGUMENT, "null argument");
    VR_HIP(hipSetDevice(device));
    const int e = vr::launch_tonemap(state, 1, pixel_count, rgb_out, stream);
    if (e) return fail(VR_ERROR_DEVICE, std::string("tonemap launch failed: ") + hipGetErrorString((hipError_t)e));
    return VR_OK;
}

int vr_tone_map(const double* colour, uint64_t pixel_count, uint8_t* rgb_out, int device) {
    if (!colour || !rgb_out) return fail(VR_ERROR_INVALID_ARGUMENT, "null argument");
    if (pixel_count == 0) return VR_OK;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(VR_ERROR_NO_DEVICE, "no HIP device");
    if (device < 0 || device >= n) return fail(VR_ERROR_INVALID_ARGUMENT, "device out of range");
    VR_HIP(hipSetDevice(device));
    CallScratch cs;
    VR_HIP(hipStreamCreateWithFlags(&cs.stream, hipStreamNonBlocking));
    const size_t in_b = (size_t)pixel_count * 3 * sizeof(double), out_b = (size_t)pixel_count * 3;
    VR_HIP(hipMalloc(&cs.ptr, in_b + out_b));
    double* d_in = (double*)cs.ptr;
    uint8_t* d_out = (uint8_t*)cs.ptr + in_b;
    VR_HIP(hipMemcpyAsync(d_in, colour, in_b, hipMemcpyHostToDevice, cs.stream));
    const int e = vr::launch_tonemap(d_in, 0, pixel_count, d_out, cs.stream);
    if (e) return fail(VR_ERROR_DEVICE, std::string("tonemap launch failed: ") + hipGetErrorString((hipError_t)e));
    VR_HIP(hipMemcpyAsync(rgb_out, d_out, out_b, hipMemcpyDeviceToHost, cs.stream));
    VR_HIP(hipStreamSynchronize(cs.stream));
    return VR_OK;
}

namespace {
void png_chunk(std::vector<uint8_t>& out, const char type[4], const uint8_t* data, size_t n) {
    const uint8_t len[4] = {(uint8_t)(n >> 24), (uint8_t)(n >> 16), (uint8_t)(n >> 8), (uint8_t)n};
    out.insert(out.end(), len, len + 4);
    const size_t at = out.size();
    out.insert(out.end(), type, type + 4);
    if (n) out.insert(out.end(), data, data + n);
    const uLong crc = crc32(0L, out.data() + at, (uInt)(4 + n));
    const uint8_t c[4] = {(uint8_t)(crc >> 24), (uint8_t)(crc >> 16), (uint8_t)(crc >> 8), (uint8_t)crc};
    out.insert(out.end(), c, c + 4);
}
}  // namespace

int vr_write_png(const char* path, const uint8_t* rgb, uint32_t width, uint32_t height) {
    if (!path || (!rgb && width && height)) return fail(VR_ERROR_INVALID_ARGUMENT, "null argument");
    if (width == 0 || height == 0) return fail(VR_ERROR_INVALID_ARGUMENT, "empty image");
    // 8-bit RGB, no interlace; every scanline carries filter type 0 (the pixels are what the
    // reference's png encoder stores -- its filter choice and compressed bytes may differ)
    const size_t row = (size_t)width * 3;
    std::vector<uint8_t> raw((row + 1) * height);
    for (uint32_t y = 0; y < height; ++y) {
        raw[y * (row + 1)] = 0;
        std::memcpy(&raw[y * (row + 1) + 1], rgb + (size_t)y * row, row);
    }
    uLongf zn = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zn);
    if (compress2(z.data(), &zn, raw.data(), (uLong)raw.size(), 6) != Z_OK) return fail(VR_ERROR_IO, "deflate failed");
    std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    const uint8_t ihdr[13] = {(uint8_t)(width >> 24), (uint8_t)(width >> 16), (uint8_t)(width >> 8), (uint8_t)width,
                              (uint8_t)(height >> 24), (uint8_t)(height >> 16), (uint8_t)(height >> 8), (uint8_t)height,
                              8, 2, 0, 0, 0};
    png_chunk(out, "IHDR", ihdr, 13);
    png_chunk(out, "IDAT", z.data(), zn);
    png_chunk(out, "IEND", nullptr, 0);
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(VR_ERROR_IO, std::string("cannot create ") + path);
    const size_t w = std::fwrite(out.data(), 1, out.size(), f);
    const int c = std::fclose(f);
    if (w != out.size() || c != 0) return fail(VR_ERROR_IO, std::string("write failed: ") + path);
    return VR_OK;
}

#ifdef VR_SPLIT_PROBE
// Analysis builds only (-DVR_SPLIT_PROBE; tools/split_probe.py, DESIGN.md section 6 "the megakernel
// split").  vr_probe_set_dump: every later render launch appends each ray it traces (origin,
// direction: 6 f64) to the device buffer `rays` (at most `cap`; *count, a device counter, takes the
// number of rays met); null turns the dump off.  vr_probe_trace: the traversal-only TRACE
// instantiation of the render kernel over n device rays, closest hits (distance; object << 32 |
// index << 2 | kind) into `hits`, at `minw` waves per SIMD and `per_cu` workgroups per CU, 16-bit
// stack entries when s16; *ms: the kernel's HIP-event time.
int vr_probe_set_dump(double* rays, unsigned long long* count, uint64_t cap) {
    g_probe.rays = rays;
    g_probe.count = count;
    g_probe.cap = rays ? cap : 0;
    return VR_OK;
}

int vr_probe_trace(const vr_scene* s, const double* rays, uint64_t n, double* hits, int minw, int s16, int per_cu,
                   void* stream, float* ms) {
    if (!s || !rays || !hits) return fail(VR_ERROR_INVALID_ARGUMENT, "null argument");
    if (s16 && s->wide_count >= 65536) return fail(VR_ERROR_UNSUPPORTED, "16-bit stack entries need < 65536 wide nodes");
    VR_HIP(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)stream;
    static unsigned long long* q = nullptr;
    static int32_t* err = nullptr;
    if (!q) VR_HIP(hipMalloc(&q, 256));
    if (!err) VR_HIP(hipMalloc(&err, 256));
    vr_render_params p{};
    p.tile.end_column = 1;
    p.tile.end_row = 1;
    p.width = p.height = 1;
    p.spp = 1;
    vr::RenderArgs a = make_args(s, &p, nullptr);
    a.probe_rays = rays;
    a.probe_hits = hits;
    a.probe_n = n;
    a.probe_count = nullptr;
    a.grab = 512;
    a.queue = q;
    a.error_flag = err;
    VR_HIP(hipMemsetAsync(q, 0, 256, st));
    VR_HIP(hipMemsetAsync(err, 0, 256, st));
    hipEvent_t e0, e1;
    VR_HIP(hipEventCreate(&e0));
    VR_HIP(hipEventCreate(&e1));
    VR_HIP(hipEventRecord(e0, st));
    const int lr = vr::launch_trace_probe(a, wide_stack_depth(s), minw, s16 != 0, std::max(1, s->cu_count) * per_cu, st);
    VR_HIP(hipEventRecord(e1, st));
    VR_HIP(hipEventSynchronize(e1));
    float t = 0.f;
    VR_HIP(hipEventElapsedTime(&t, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (lr) return fail(VR_ERROR_UNSUPPORTED, "no TRACE instantiation for this stack / waves choice");
    if (ms) *ms = t;
    return VR_OK;
}
#endif
}  // extern "C"

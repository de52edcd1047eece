// vr_qnode.h -- quantisation of a 4-wide node's child boxes to the 64-B Node4q (vr_layout.h).
//
// Host and device code (the device fills the array after the 4-wide tree exists on the GPU,
// vr_build.hip quantize_wide_kernel; the host exports the same function for the CPU soundness test,
// vr_quantize_wide_node).  All arithmetic that decides a plane is exact: the grid step is a power of
// two, q * 2^e is exact, and origin + q * 2^e is compared with the f32 plane through an exact
// two-sum, so every decoded lower plane is <= the f32 lower plane and every upper plane >= the f32
// upper plane.  The f32 planes are already rounded outward from the f64 boxes (Node4), so the decoded
// box contains the child's f64 box.
#pragma once

#include <math.h>
#include <stdint.h>

#include "vr_layout.h"

#if defined(__HIPCC__) || defined(__HIP__)
#define VR_HD __host__ __device__
#else
#define VR_HD
#endif

namespace vr {

// origin + q * s <= x exactly (s a power of two, q an integer <= 255: q * s exact; the sum as an f64
// two-sum, whose (sum, err) pair represents origin + q * s exactly when no term overflows)
VR_HD inline bool q_plane_le(double origin, double q, double s, double x) {
    const double b = q * s;
    const double sum = origin + b;
    const double bv = sum - origin;
    const double err = (origin - (sum - bv)) + (b - bv);
    return sum < x || (sum == x && err <= 0.0);
}
VR_HD inline bool q_plane_ge(double origin, double q, double s, double x) {
    const double b = q * s;
    const double sum = origin + b;
    const double bv = sum - origin;
    const double err = (origin - (sum - bv)) + (b - bv);
    return sum > x || (sum == x && err >= 0.0);
}

// Quantises w's live children (child != kEmptyChild) into out.  Returns false -- out unusable --
// when a live child's box is not finite (the scene then keeps the 128-B nodes).
VR_HD inline bool quantize_node4(const Node4& w, Node4q& out) {
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    int live = 0;
    for (int k = 0; k < 4; ++k) {
        out.child[k] = w.child[k];
        if (w.child[k] == kEmptyChild) continue;
        ++live;
        for (int a = 0; a < 3; ++a) {
            const double l = w.box[k][2 * a], h = w.box[k][2 * a + 1];
            if (!(fabs(l) <= 3.0e38) || !(fabs(h) <= 3.0e38)) return false;
            lo[a] = l < lo[a] ? l : lo[a];
            hi[a] = h > hi[a] ? h : hi[a];
        }
    }
    out.pad0 = 0;
    out.pad1[0] = out.pad1[1] = 0;
    for (int j = 0; j < 6; ++j) out.q[j] = 0;
    if (!live) {
        for (int a = 0; a < 3; ++a) {
            out.origin[a] = 0.0f;
            out.exp[a] = 0;
        }
        return true;
    }
    for (int a = 0; a < 3; ++a) {
        // the grid: origin = the children's lowest plane (an f32 value), step 2^e with 255 steps
        // reaching the highest plane (e >= -126: a normal step, and |S| = 2^e |1 / d| stays normal
        // for a normalised direction, whose reciprocals are >= 1 in magnitude)
        const double o = lo[a];
        const double span = hi[a] - o;  // f64: exact for f32 operands of moderate exponent spread
        int e = -126;
        while (e < 127 && !(255.0 * ldexp(1.0, e) >= span)) ++e;
        const double s = ldexp(1.0, e);
        // 255 * s >= span as computed; make it exact: the top plane must reach hi
        while (e < 127 && !q_plane_ge(o, 255.0, s, hi[a])) ++e;
        if (!q_plane_ge(o, 255.0, ldexp(1.0, e), hi[a])) return false;
        out.origin[a] = (float)o;  // exact: o is one of the f32 planes
        out.exp[a] = (int8_t)e;
        const double st = ldexp(1.0, e);
        for (int k = 0; k < 4; ++k) {
            if (w.child[k] == kEmptyChild) continue;
            const double l = w.box[k][2 * a], h = w.box[k][2 * a + 1];
            // lower plane: the largest q with origin + q s <= l; upper: the smallest with >= h
            double ql = floor((l - o) / st);
            ql = ql < 0.0 ? 0.0 : (ql > 255.0 ? 255.0 : ql);
            while (ql > 0.0 && !q_plane_le(o, ql, st, l)) ql -= 1.0;
            while (ql < 255.0 && q_plane_le(o, ql + 1.0, st, l)) ql += 1.0;
            double qh = ceil((h - o) / st);
            qh = qh < 0.0 ? 0.0 : (qh > 255.0 ? 255.0 : qh);
            while (qh < 255.0 && !q_plane_ge(o, qh, st, h)) qh += 1.0;
            while (qh > 0.0 && q_plane_ge(o, qh - 1.0, st, h)) qh -= 1.0;
            if (!q_plane_le(o, ql, st, l) || !q_plane_ge(o, qh, st, h)) return false;
            out.q[2 * a] |= (uint32_t)ql << (8 * k);
            out.q[2 * a + 1] |= (uint32_t)qh << (8 * k);
        }
    }
    return true;
}

}  // namespace vr

#undef VR_HD

// vr_image.hip -- the display end of the path on the device: the accumulation buffer's CIE XYZ
// colour to 8-bit sRGB (ClampingToneMapper, src/image.rs:166-187, over ColourXyz::to_srgb,
// src/colour/colour_xyz.rs:49-84), and ImageRgbU8::write_png (src/image.rs:52-66) on the host.
//
// One thread per pixel; the kernel reads 24 B (colour) or 64 B (device records) and writes 3 B
// per pixel, so it is HBM-bound: 1024^2 pixels move 70 MB (records), about 10 us at 8 TB/s.
// Compiled with -ffp-contract=off like the render kernel: the 3x3 transform is three dot
// products folded from -0.0 in the reference's order (mat3.rs:147-157, vec3.rs:76-82).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "vr_layout.h"

namespace vr {
namespace dev {

// srgb_gamma with the reference's constants (colour_xyz.rs:78-84; 12.98 and 1.005 are not the
// sRGB standard's 12.92 / 1.055 -- kept as written)
__device__ __forceinline__ double srgb_gamma(double u) {
    if (u <= 0.0031308) return 12.98 * u;
    return 1.005 * pow(u, 1.0 / 2.4) - 0.055;
}

// ClampingToneMapper::clamp + NormalizedAsByte for f64 (image.rs:110-128,141-145):
// f64::clamp(0, 1) keeps NaN, and Rust's saturating `as u8` maps NaN to 0
__device__ __forceinline__ uint8_t to_byte(double v) {
    if (v != v) return 0;
    const double c = v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v);
    return (uint8_t)(c * 255.0);  // c * 255 in [0, 255]: truncation toward zero
}

__device__ __forceinline__ double dot_m0(double a, double b, double c, double x, double y, double z) {
    double s = -0.0;  // Sum for f64 folds from -0.0
    s = s + a * x;
    s = s + b * y;
    s = s + c * z;
    return s;
}

// `src` = device records (vr_layout.h: npix x {sum X, Y, Z, weight}, then the compensations;
// colour = colour_sum * (1 / weight), 0 where no sample landed, as AccumulationBuffer::new leaves
// it) or 3 f64 per pixel (the colour buffer)
__global__ __launch_bounds__(256) void tonemap_kernel(const double* src, int from_state, uint64_t npix,
                                                      uint8_t* rgb) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= npix) return;
    double x, y, z;
    if (from_state) {
        const double* r = src + 4 * p;
        const double w = r[3];
        const double inv = 1.0 / w;
        x = w != 0.0 ? r[0] * inv : 0.0;
        y = w != 0.0 ? r[1] * inv : 0.0;
        z = w != 0.0 ? r[2] * inv : 0.0;
    } else {
        x = src[3 * p];
        y = src[3 * p + 1];
        z = src[3 * p + 2];
    }
    // ColourXyz::to_linear_rgb (colour_xyz.rs:49-56)
    const double r = dot_m0(3.24096994, -1.53738318, -0.49861076, x, y, z);
    const double g = dot_m0(-0.96924364, 1.87596750, 0.04155506, x, y, z);
    const double b = dot_m0(0.05563008, -0.20397696, 1.05697151, x, y, z);
    rgb[3 * p] = to_byte(srgb_gamma(r));
    rgb[3 * p + 1] = to_byte(srgb_gamma(g));
    rgb[3 * p + 2] = to_byte(srgb_gamma(b));
}

}  // namespace dev

namespace dev {
// Host AccumulationBuffer layout (accumulation_buffer.rs:6-12, include/vanrijn_amd.h) <-> the
// device records (vr_layout.h: sums {X, Y, Z, weight} of every pixel, then their compensations).  planar = [colour 3n | colour_sum 3n | colour_bias 3n |
// weight n | weight_bias n] doubles, so one host array is one contiguous copy.
__global__ __launch_bounds__(256) void export_buffer_kernel(const double* __restrict__ state, uint64_t npix,
                                                            double* __restrict__ planar) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= npix) return;
    const double* r = state + p * 4;
    const double* b = state + 4 * npix + p * 4;
    const double w = r[3];
    const double inv = 1.0 / w;  // accumulation_buffer.rs:59: colour = sum * (1 / weight)
    for (int k = 0; k < 3; ++k) {
        planar[3 * p + k] = w != 0.0 ? r[k] * inv : 0.0;
        planar[3 * npix + 3 * p + k] = r[k];
        planar[6 * npix + 3 * p + k] = b[k];
    }
    planar[9 * npix + p] = w;
    planar[10 * npix + p] = b[3];
}
// A fresh buffer after exactly one sample per pixel (vr_partial_render_scene): weight 1, weight
// bias 0, and colour / colour_bias follow from colour_sum alone, so only the sums cross PCIe
// (24 of the 88 B per pixel); the host expands them (vr_host.cpp expand_fresh_one_sample).
__global__ __launch_bounds__(256) void export_sums_kernel(const double* __restrict__ state, uint64_t npix,
                                                          double* __restrict__ sums) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= npix) return;
    const double* r = state + p * 4;
    for (int k = 0; k < 3; ++k) sums[3 * p + k] = r[k];
}
__global__ __launch_bounds__(256) void import_buffer_kernel(const double* __restrict__ planar, uint64_t npix,
                                                            double* __restrict__ state) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= npix) return;
    double* r = state + p * 4;
    double* b = state + 4 * npix + p * 4;
    for (int k = 0; k < 3; ++k) {
        r[k] = planar[3 * npix + 3 * p + k];
        b[k] = planar[6 * npix + 3 * p + k];
    }
    r[3] = planar[9 * npix + p];
    b[3] = planar[10 * npix + p];
}
}  // namespace dev

int launch_buffer_convert(const double* src, double* dst, uint64_t npix, int to_planar, void* stream) {
    if (npix == 0) return 0;
    const dim3 grid((unsigned)((npix + 255) / 256)), block(256);
    if (to_planar == 2) hipLaunchKernelGGL(dev::export_sums_kernel, grid, block, 0, (hipStream_t)stream, src, npix, dst);
    else if (to_planar) hipLaunchKernelGGL(dev::export_buffer_kernel, grid, block, 0, (hipStream_t)stream, src, npix, dst);
    else hipLaunchKernelGGL(dev::import_buffer_kernel, grid, block, 0, (hipStream_t)stream, src, npix, dst);
    return (int)hipGetLastError();
}

int launch_tonemap(const double* src, int from_state, uint64_t npix, uint8_t* rgb, void* stream) {
    if (npix == 0) return 0;
    hipLaunchKernelGGL(dev::tonemap_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, src, from_state, npix, rgb);
    return (int)hipGetLastError();
}

}  // namespace vr

// opcost.hip -- measured issue cost of the render kernel's dominant VALU opcodes on gfx950.
//
// The roofline's VALU-issue bound prices the kernel's instruction mix (rocprofv3 PMC classes) at
// a per-instruction issue cost.  MI355X_MICROARCH.md gives f32 costs only (v_fma_f32: 2 cycles
// per wave64 instruction on a SIMD, 4 for one wave alone), so this program measures the f64,
// 64-bit integer and compare / select opcodes the kernel issues (tools/isa_sections.py's static
// mix) the same way: each wave runs a loop of 32 independent instructions of one opcode (8
// accumulators x 4), and the SIMD's cycles per instruction are
//     (the SIMD's busy span in shader cycles: first wave start .. last wave end, s_memtime)
//     / (instructions per wave x waves sharing the SIMD),
// the median over the chip's SIMDs (a wave's own lifetime undercounts when the waves of a SIMD do
// not start together).
// Occupancy is forced by LDS: a 256-thread workgroup (4 waves, one per SIMD) reserves 96 / 64 /
// 48 / 36 KB, so exactly 1 / 2 / 3 / 4 workgroups fit a CU's 160 KB, and the grid is that many
// workgroups per CU; every wave also records its hardware id (CU, SIMD, XCC), and the host checks
// that each SIMD held the intended number of waves.
//   hipcc --offload-arch=gfx950 -O3 tools/opcost.hip -o tools/opcost && tools/opcost > opcost.json
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <tuple>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

// one opcode over 8 independent accumulators; R4 repeats it 4 times (32 per loop iteration)
#define R4(x) x x x x
#define D8(op) \
    R4(op(0) op(1) op(2) op(3) op(4) op(5) op(6) op(7))

enum Op {
    kAddF64, kMulF64, kFmaF64, kMaxF64, kMinF64, kRcpF64, kSqrtF64, kRsqF64, kDivScaleF64, kDivFmasF64,
    kDivFixupF64, kCmpF64, kFractF64, kLdexpF64, kCvtF64I32, kCvtF32F64, kAddF32, kFmaF32, kPkFmaF32,
    kCndmask, kAddU32, kMulLoU32, kLshl64, kMadU64U32, kAdd64, kBfeU32, kCndmaskE64, kMovB32, kXorB32,
    kMaxF32, kCmpF32, kCmpU32, kMulF32, kCndmaskE64Vcc, kCndmaskSaluVcc, kCndmaskE32Fresh, kFmacF64,
    kCndmaskE32Mixed, kNumOps
};
static const char* kNames[kNumOps] = {
    "v_add_f64", "v_mul_f64", "v_fma_f64", "v_max_f64", "v_min_f64", "v_rcp_f64", "v_sqrt_f64", "v_rsq_f64",
    "v_div_scale_f64", "v_div_fmas_f64", "v_div_fixup_f64", "v_cmp_lt_f64", "v_fract_f64", "v_ldexp_f64",
    "v_cvt_f64_i32", "v_cvt_f32_f64", "v_add_f32", "v_fma_f32", "v_pk_fma_f32", "v_cndmask_b32", "v_add_u32",
    "v_mul_lo_u32", "v_lshlrev_b64", "v_mad_u64_u32", "v_add_co_u32+v_addc_co_u32 (one 64-bit add)", "v_bfe_u32",
    "v_cndmask_b32_e64 (sgpr mask)", "v_mov_b32", "v_xor_b32", "v_max_f32", "v_cmp_lt_f32", "v_cmp_lt_u32", "v_mul_f32",
    "v_cndmask_b32_e64 (vcc operand)", "v_cndmask_b32 (vcc from s_mov_b64)", "v_cndmask_b32 (e32, fresh destination)",
    "v_fmac_f64", "v_cndmask_b32 (e32) + v_add_u32 interleaved (pair)"};

template <int OP>
__device__ __forceinline__ void body(double (&d)[8], float (&f)[8], unsigned (&u)[8], unsigned (&w)[8],
                                     unsigned long long (&q)[8], double db, float fb, unsigned ub) {
    // each asm block: 32 instructions (the 64-bit add: 32 pairs, counted as 32 "instructions")
#define ASM_D(i) asm volatile(OPSTR : "+v"(d[i]) : "v"(db));
    if constexpr (OP == kAddF64) {
#define OPSTR "v_add_f64 %0, %0, %1"
        D8(ASM_D)
#undef OPSTR
    } else if constexpr (OP == kMulF64) {
#define OPSTR "v_mul_f64 %0, %0, %1"
        D8(ASM_D)
#undef OPSTR
    } else if constexpr (OP == kFmaF64) {
#define OPSTR "v_fma_f64 %0, %0, %1, %1"
        D8(ASM_D)
#undef OPSTR
    } else if constexpr (OP == kMaxF64) {
#define OPSTR "v_max_f64 %0, %0, %1"
        D8(ASM_D)
#undef OPSTR
    } else if constexpr (OP == kMinF64) {
#define OPSTR "v_min_f64 %0, %0, %1"
        D8(ASM_D)
#undef OPSTR
    } else if constexpr (OP == kRcpF64) {
#define OPSTR "v_rcp_f64 %0, %0"
        D8(ASM_D)
#undef OPSTR
    } else if constexpr (OP == kSqrtF64) {
#define OPSTR "v_sqrt_f64 %0, %0"
        D8(ASM_D)
#undef OPSTR
    } else if constexpr (OP == kRsqF64) {
#define OPSTR "v_rsq_f64 %0, %0"
        D8(ASM_D)
#undef OPSTR
    } else if constexpr (OP == kDivScaleF64) {
#define ASM_DS(i) asm volatile("v_div_scale_f64 %0, vcc, %0, %1, %0" : "+v"(d[i]) : "v"(db) : "vcc");
        D8(ASM_DS)
#undef ASM_DS
    } else if constexpr (OP == kDivFmasF64) {
#define OPSTR "v_div_fmas_f64 %0, %0, %1, %1"
        D8(ASM_D)
#undef OPSTR
    } else if constexpr (OP == kDivFixupF64) {
#define OPSTR "v_div_fixup_f64 %0, %0, %1, %1"
        D8(ASM_D)
#undef OPSTR
    } else if constexpr (OP == kCmpF64) {
#define ASM_C(i) asm volatile("v_cmp_lt_f64_e64 %0, %1, %2" : "=s"(q[i]) : "v"(d[i]), "v"(db));
        D8(ASM_C)
#undef ASM_C
    } else if constexpr (OP == kFractF64) {
#define OPSTR "v_fract_f64 %0, %0"
        D8(ASM_D)
#undef OPSTR
    } else if constexpr (OP == kLdexpF64) {
#define ASM_L(i) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d[i]) : "v"(ub));
        D8(ASM_L)
#undef ASM_L
    } else if constexpr (OP == kCvtF64I32) {
#define ASM_CV(i) asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(d[i]) : "v"(u[i]));
        D8(ASM_CV)
#undef ASM_CV
    } else if constexpr (OP == kCvtF32F64) {
#define ASM_CV(i) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f[i]) : "v"(d[i]));
        D8(ASM_CV)
#undef ASM_CV
    } else if constexpr (OP == kAddF32) {
#define ASM_F(i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[i]) : "v"(fb));
        D8(ASM_F)
#undef ASM_F
    } else if constexpr (OP == kFmaF32) {
#define ASM_F(i) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[i]) : "v"(fb));
        D8(ASM_F)
#undef ASM_F
    } else if constexpr (OP == kPkFmaF32) {
        // packed: two f32 in a 64-bit register pair (the node step's slab32 tests)
#define ASM_P(i) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(d[i]) : "v"(db));
        D8(ASM_P)
#undef ASM_P
    } else if constexpr (OP == kCndmask) {
#define ASM_S(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(ub));
        D8(ASM_S)
#undef ASM_S
    } else if constexpr (OP == kAddU32) {
#define ASM_U(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(ub));
        D8(ASM_U)
#undef ASM_U
    } else if constexpr (OP == kMulLoU32) {
#define ASM_U(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[i]) : "v"(ub));
        D8(ASM_U)
#undef ASM_U
    } else if constexpr (OP == kLshl64) {
#define ASM_Q(i) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(q[i]));
        D8(ASM_Q)
#undef ASM_Q
    } else if constexpr (OP == kMadU64U32) {
#define ASM_Q(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(q[i]) : "v"(ub) : "vcc");
        D8(ASM_Q)
#undef ASM_Q
    } else if constexpr (OP == kAdd64) {
#define ASM_Q(i) \
    asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, 0, vcc" : "+v"(u[i]), "+v"(w[i]) : "v"(ub) : "vcc");
        D8(ASM_Q)
#undef ASM_Q
    } else if constexpr (OP == kBfeU32) {
#define ASM_U(i) asm volatile("v_bfe_u32 %0, %0, 3, 7" : "+v"(u[i]));
        D8(ASM_U)
#undef ASM_U
    } else if constexpr (OP == kCndmaskE64) {
#define ASM_S(i) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(u[i]) : "v"(ub), "s"(0x5555555555555555ull));
        D8(ASM_S)
#undef ASM_S
    } else if constexpr (OP == kMovB32) {
#define ASM_U(i) asm volatile("v_mov_b32 %0, %1" : "=v"(u[i]) : "v"(w[i]));
        D8(ASM_U)
#undef ASM_U
    } else if constexpr (OP == kXorB32) {
#define ASM_U(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u[i]) : "v"(ub));
        D8(ASM_U)
#undef ASM_U
    } else if constexpr (OP == kMaxF32) {
#define ASM_F(i) asm volatile("v_max_f32 %0, %0, %1" : "+v"(f[i]) : "v"(fb));
        D8(ASM_F)
#undef ASM_F
    } else if constexpr (OP == kCmpF32) {
#define ASM_C(i) asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "=s"(q[i]) : "v"(f[i]), "v"(fb));
        D8(ASM_C)
#undef ASM_C
    } else if constexpr (OP == kCmpU32) {
#define ASM_C(i) asm volatile("v_cmp_lt_u32_e64 %0, %1, %2" : "=s"(q[i]) : "v"(u[i]), "v"(ub));
        D8(ASM_C)
#undef ASM_C
    } else if constexpr (OP == kMulF32) {
#define ASM_F(i) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(f[i]) : "v"(fb));
        D8(ASM_F)
#undef ASM_F
    } else if constexpr (OP == kCndmaskE64Vcc) {
#define ASM_S(i) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(ub));
        D8(ASM_S)
#undef ASM_S
    } else if constexpr (OP == kCndmaskSaluVcc) {
        // vcc written by the scalar unit (no VALU-written lane mask in flight)
        asm volatile("s_mov_b64 vcc, 0x5555" ::: "vcc");
#define ASM_S(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(ub));
        D8(ASM_S)
#undef ASM_S
    } else if constexpr (OP == kCndmaskE32Fresh) {
#define ASM_S(i) asm volatile("v_cndmask_b32 %0, %1, %2, vcc" : "=v"(u[i]) : "v"(w[i]), "v"(ub));
        D8(ASM_S)
#undef ASM_S
    } else if constexpr (OP == kFmacF64) {
#define ASM_D2(i) asm volatile("v_fmac_f64 %0, %1, %1" : "+v"(d[i]) : "v"(db));
        D8(ASM_D2)
#undef ASM_D2
    } else if constexpr (OP == kCndmaskE32Mixed) {
#define ASM_S(i) asm volatile("v_cndmask_b32 %0, %0, %2, vcc\n\tv_add_u32 %1, %1, %2" : "+v"(u[i]), "+v"(w[i]) : "v"(ub));
        D8(ASM_S)
#undef ASM_S
    }
#undef ASM_D
}

template <int OP, int LDS>
__global__ __launch_bounds__(256) void opk(int iters, unsigned long long* out, double* sink) {
    __shared__ char pad[LDS];
    const int tid = threadIdx.x;
    pad[tid] = (char)tid;  // the reservation must survive optimisation
    __syncthreads();
    double d[8];
    float f[8];
    unsigned u[8], w[8];
    unsigned long long q[8];
    for (int i = 0; i < 8; ++i) {
        d[i] = 1.0 + 1e-9 * (tid + i);
        f[i] = 1.0f + 1e-6f * (float)(tid + i);
        u[i] = (unsigned)(tid * 8 + i + 1);
        w[i] = (unsigned)i;
        q[i] = 0x123456789ull + tid + i;
    }
    const double db = 0.9999999999 + 1e-12 * pad[(tid + 1) & 255];
    const float fb = 0.99999f;
    const unsigned ub = 3u + (unsigned)pad[(tid + 2) & 255];
    asm volatile("v_cmp_lt_f64 vcc, %0, %1" ::"v"(d[0]), "v"(db) : "vcc");  // vcc for div_fmas / cndmask
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) body<OP>(d, f, u, w, q, db, fb, ub);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    double acc = 0.0;
    for (int i = 0; i < 8; ++i) acc += d[i] + (double)f[i] + (double)u[i] + (double)w[i] + (double)q[i];
    sink[blockIdx.x * 256 + tid] = acc;  // keeps every result live
    if ((tid & 63) == 0) {
        unsigned long long* o = out + 5 * (blockIdx.x * 4 + (tid >> 6));
        o[0] = t0;
        o[1] = t1;
        o[4] = r1 - r0;
        o[2] = hw;
        o[3] = xcc;
    }
}

template <int OP>
static void launch(int k, int grid, int iters, unsigned long long* out, double* sink) {
    switch (k) {
        case 1: hipLaunchKernelGGL((opk<OP, 98304>), dim3(grid), dim3(256), 0, 0, iters, out, sink); break;
        case 2: hipLaunchKernelGGL((opk<OP, 65536>), dim3(grid), dim3(256), 0, 0, iters, out, sink); break;
        case 3: hipLaunchKernelGGL((opk<OP, 49152>), dim3(grid), dim3(256), 0, 0, iters, out, sink); break;
        default: hipLaunchKernelGGL((opk<OP, 36864>), dim3(grid), dim3(256), 0, 0, iters, out, sink); break;
    }
}

template <int OP = 0>
static void launch_op(int op, int k, int grid, int iters, unsigned long long* out, double* sink) {
    if constexpr (OP < kNumOps) {
        if (op == OP) launch<OP>(k, grid, iters, out, sink);
        else launch_op<OP + 1>(op, k, grid, iters, out, sink);
    }
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2048;
    const char* only = argc > 2 ? argv[2] : nullptr;  // substring filter on the opcode names
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int max_grid = cus * 4;
    unsigned long long* d_out = nullptr;
    double* d_sink = nullptr;
    CHECK(hipMalloc(&d_out, sizeof(unsigned long long) * 5 * 4 * max_grid));
    CHECK(hipMalloc(&d_sink, sizeof(double) * 256 * max_grid));
    std::vector<unsigned long long> h(5 * 4 * max_grid);
    std::printf("{\"device_cus\": %d, \"iters\": %d, \"insts_per_wave\": %d, \"results\": [\n", cus, iters, iters * 32);
    bool first = true;
    for (int op = 0; op < kNumOps; ++op) {
        if (only && !std::strstr(kNames[op], only)) continue;
        for (int k = 1; k <= 4; ++k) {
            const int grid = cus * k;
            launch_op(op, k, grid, iters / 8, d_out, d_sink);  // warm-up (clocks, code fetch)
            CHECK(hipDeviceSynchronize());
            launch_op(op, k, grid, iters, d_out, d_sink);
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(h.data(), d_out, sizeof(unsigned long long) * 5 * 4 * grid, hipMemcpyDeviceToHost));
            // per SIMD (xcc, se, cu, simd from the hardware ids): its waves and busy span
            std::map<std::tuple<unsigned, unsigned, unsigned, unsigned>, std::vector<int>> per_simd;
            std::vector<double> life, clk;
            for (int w = 0; w < 4 * grid; ++w) {
                const unsigned long long* o = &h[5 * w];
                const unsigned hw = (unsigned)o[2], xcc = (unsigned)o[3] & 0xf;
                per_simd[std::make_tuple(xcc, (hw >> 13) & 7, (hw >> 8) & 15, (hw >> 4) & 3)].push_back(w);
                life.push_back((double)(o[1] - o[0]));
                clk.push_back((double)(o[1] - o[0]) / ((double)o[4] / 100.0));  // MHz (memrealtime: 100 MHz)
            }
            int lo = 1 << 30, hi = 0;
            std::vector<double> cpi;
            for (auto& kv : per_simd) {
                lo = std::min(lo, (int)kv.second.size());
                hi = std::max(hi, (int)kv.second.size());
                unsigned long long t0 = ~0ull, t1 = 0;
                for (int w : kv.second) {
                    t0 = std::min(t0, h[5 * w]);
                    t1 = std::max(t1, h[5 * w + 1]);
                }
                cpi.push_back((double)(t1 - t0) / ((double)iters * 32.0 * (double)kv.second.size()));
            }
            std::sort(cpi.begin(), cpi.end());
            std::sort(life.begin(), life.end());
            std::sort(clk.begin(), clk.end());
            std::printf("%s  {\"op\": \"%s\", \"waves_per_simd\": %d, \"simds\": %zu, \"waves_per_simd_min\": %d, "
                        "\"waves_per_simd_max\": %d, \"cycles_per_inst\": %.3f, \"cycles_per_inst_p10\": %.3f, "
                        "\"cycles_per_inst_p90\": %.3f, \"wave_lifetime_median\": %.0f, \"clock_mhz_median\": %.0f}",
                        first ? "" : ",\n", kNames[op], k, per_simd.size(), lo, hi, cpi[cpi.size() / 2],
                        cpi[cpi.size() / 10], cpi[cpi.size() * 9 / 10], life[life.size() / 2], clk[clk.size() / 2]);
            first = false;
        }
    }
    std::printf("\n]}\n");
    CHECK(hipFree(d_out));
    CHECK(hipFree(d_sink));
    return 0;
}

/* vr_exp_table.h -- exp(x) for x in [-745, 0] by a 64-entry table of 2^(j/64): the ordered reduce's
 * CIE lobes (7 exp per sample).  x = (64 m + j) ln2/64 + r, |r| <= ln2/128 (Cody-Waite with a
 * 36-bit ln2/64, so n * hi is exact for |n| < 2^17); e^r - 1 by its degree-6 Taylor polynomial
 * (truncation < 3e-20); result 2^m * T[j] * (1 + p).  Within 2 ulp of exp (tests/test_exp_table.py
 * compiles this header with gcc and checks 10^7 arguments against libm); 13 VALU operations
 * instead of the general exp's 22.  Plain C99 so the test builds it unchanged.
 * Table: correctly rounded 2^(j/64), j = 0..63 (decimal arithmetic at 60 digits). */
#ifndef VR_EXP_TABLE_H
#define VR_EXP_TABLE_H

#include <math.h>

#ifdef __HIPCC__
#define VR_EXP_FN __host__ __device__ static inline
#else
#define VR_EXP_FN static inline
#endif

#define VR_EXP_TABLE_INIT { \
    0x1.0000000000000p+0, 0x1.02c9a3e778061p+0, 0x1.059b0d3158574p+0, 0x1.0874518759bc8p+0, \
    0x1.0b5586cf9890fp+0, 0x1.0e3ec32d3d1a2p+0, 0x1.11301d0125b51p+0, 0x1.1429aaea92de0p+0, \
    0x1.172b83c7d517bp+0, 0x1.1a35beb6fcb75p+0, 0x1.1d4873168b9aap+0, 0x1.2063b88628cd6p+0, \
    0x1.2387a6e756238p+0, 0x1.26b4565e27cddp+0, 0x1.29e9df51fdee1p+0, 0x1.2d285a6e4030bp+0, \
    0x1.306fe0a31b715p+0, 0x1.33c08b26416ffp+0, 0x1.371a7373aa9cbp+0, 0x1.3a7db34e59ff7p+0, \
    0x1.3dea64c123422p+0, 0x1.4160a21f72e2ap+0, 0x1.44e086061892dp+0, 0x1.486a2b5c13cd0p+0, \
    0x1.4bfdad5362a27p+0, 0x1.4f9b2769d2ca7p+0, 0x1.5342b569d4f82p+0, 0x1.56f4736b527dap+0, \
    0x1.5ab07dd485429p+0, 0x1.5e76f15ad2148p+0, 0x1.6247eb03a5585p+0, 0x1.6623882552225p+0, \
    0x1.6a09e667f3bcdp+0, 0x1.6dfb23c651a2fp+0, 0x1.71f75e8ec5f74p+0, 0x1.75feb564267c9p+0, \
    0x1.7a11473eb0187p+0, 0x1.7e2f336cf4e62p+0, 0x1.82589994cce13p+0, 0x1.868d99b4492edp+0, \
    0x1.8ace5422aa0dbp+0, 0x1.8f1ae99157736p+0, 0x1.93737b0cdc5e5p+0, 0x1.97d829fde4e50p+0, \
    0x1.9c49182a3f090p+0, 0x1.a0c667b5de565p+0, 0x1.a5503b23e255dp+0, 0x1.a9e6b5579fdbfp+0, \
    0x1.ae89f995ad3adp+0, 0x1.b33a2b84f15fbp+0, 0x1.b7f76f2fb5e47p+0, 0x1.bcc1e904bc1d2p+0, \
    0x1.c199bdd85529cp+0, 0x1.c67f12e57d14bp+0, 0x1.cb720dcef9069p+0, 0x1.d072d4a07897cp+0, \
    0x1.d5818dcfba487p+0, 0x1.da9e603db3285p+0, 0x1.dfc97337b9b5fp+0, 0x1.e502ee78b3ff6p+0, \
    0x1.ea4afa2a490dap+0, 0x1.efa1bee615a27p+0, 0x1.f50765b6e4540p+0, 0x1.fa7c1819e90d8p+0, \
}

#define VR_EXP_INV_L 0x1.71547652b82fep+6  /* 64 / ln2 */
#define VR_EXP_L_HI 0x1.62e42fefa0000p-7   /* ln2 / 64, 36 significant bits */
#define VR_EXP_L_LO 0x1.cf79abc9e3b3ap-46  /* ln2 / 64 - VR_EXP_L_HI */

/* tab: the 64 entries of VR_EXP_TABLE_INIT (wherever the caller keeps them) */
VR_EXP_FN double vr_exp_tab(double x, const double* tab) {
    const double n = rint(x * VR_EXP_INV_L);
    const int ni = (int)n;
    const double r = fma(-n, VR_EXP_L_LO, fma(-n, VR_EXP_L_HI, x));
    const double q = fma(r, fma(r, fma(r, fma(r, 1.0 / 720.0, 1.0 / 120.0), 1.0 / 24.0), 1.0 / 6.0), 0.5);
    const double p = fma(r * r, q, r);
    const double t = tab[ni & 63];
    return ldexp(fma(t, p, t), ni >> 6);
}

#endif

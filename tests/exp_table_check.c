/* Max ulp distance of vr_exp_tab (vanrijn_amd/csrc/vr_exp_table.h) from libm exp over the reduce's
 * argument range: a deterministic sweep of [-745, 0] plus the CIE lobes' exponents at
 * wavelengths 0 and 380..740 nm.  Prints "<max ulp> <points>".  Built by tests/test_exp_table.py
 * with gcc -O2 -ffp-contract=off. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../vanrijn_amd/csrc/vr_exp_table.h"

static const double tab[64] = VR_EXP_TABLE_INIT;

static int64_t ord(double v) {
    int64_t i;
    memcpy(&i, &v, 8);
    return i < 0 ? INT64_MIN - i : i;
}

static double worst = 0.0;
static long points = 0;

static void check(double x) {
    const double a = vr_exp_tab(x, tab), b = exp(x);
    const double d = fabs((double)(ord(a) - ord(b)));
    if (d > worst) worst = d;
    ++points;
}

int main(void) {
    uint64_t s = 0x243F6A8885A308D3ull;
    for (long i = 0; i < 10000000; ++i) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        check(-745.0 * (double)(s >> 11) * 0x1.0p-53);
    }
    for (long i = 0; i < 1000000; ++i) {  /* small arguments, where r = x */
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        check(-0.02 * (double)(s >> 11) * 0x1.0p-53);
    }
    /* the reduce's exponents: -(t^2) k for the seven lobes of colour_xyz.rs:86-103 */
    static const double lobes[7][3] = {{599.8, 37.9, 31.0}, {442.0, 16.0, 26.7}, {501.1, 20.4, 26.2},
                                       {568.8, 46.9, 40.5}, {530.9, 16.3, 31.1}, {437.0, 11.8, 36.0},
                                       {459.0, 26.0, 13.8}};
    for (int k = 0; k < 7; ++k)
        for (long i = -1; i <= 3600000; ++i) {
            const double wl = i < 0 ? 0.0 : 380.0 + (double)i * 1e-4;
            const double mu = lobes[k][0], sg = wl < mu ? lobes[k][1] : lobes[k][2];
            const double t = wl - mu;
            check(-(t * t) * (1.0 / (2.0 * (sg * sg))));
        }
    check(0.0);
    check(-0.0);
    check(-745.0);
    printf("%.0f %ld\n", worst, points);
    return 0;
}

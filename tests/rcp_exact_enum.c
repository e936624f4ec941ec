/* Enumeration behind rcp_rn_mid (hello-raytracing_amd/csrc/rt_device.hpp): for every f32 significand l in [1, 2)
 * and every starting value r0 within 1 ulp of 1 / l (the two floats around it, i.e. any v_rcp_f32 result that
 * meets its 1-ulp accuracy), one Newton step r1 = fma(fma(-l, r0, 1), r0, r0) against the correctly rounded
 * 1.0f / l of the host (SSE division). Prints "cases bad" and then one line per bad case: "m r0 r1 ref" as hex
 * bit patterns. Scaling l by 2^k (|k| <= 60) scales r0, the residual and r1 exactly, so one binade covers the
 * range the kernels use; the sign is symmetric. Test infrastructure (tests/test_rcp_exact.py). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(void) {
    unsigned long cases = 0, bad = 0;
    static uint32_t rec[64][4];
    for (uint32_t m = 0; m < (1u << 23); m++) {
        const float l = u2f((127u << 23) | m);
        const float ref = 1.0f / l;
        const double x = 1.0 / (double)l; /* 53 bits: 1 / l is never within 2^-48 of a float or a midpoint */
        float rd = (float)x;
        if ((double)rd > x) rd = nextafterf(rd, 0.0f);
        /* 1 / l exact (l = 1): the float itself and both neighbours are within 1 ulp */
        const int exact = (double)rd == x;
        const float cand[3] = {exact ? nextafterf(rd, 0.0f) : rd, nextafterf(rd, 2.0f), rd};
        for (int c = 0; c < 2 + exact; c++) {
            const float r0 = cand[c];
            const float r1 = fmaf(fmaf(-l, r0, 1.0f), r0, r0);
            cases++;
            if (f2u(r1) != f2u(ref)) {
                if (bad < 64) {
                    rec[bad][0] = m; rec[bad][1] = f2u(r0); rec[bad][2] = f2u(r1); rec[bad][3] = f2u(ref);
                }
                bad++;
            }
        }
    }
    printf("%lu %lu\n", cases, bad);
    for (unsigned long i = 0; i < bad && i < 64; i++)
        printf("%06x %08x %08x %08x\n", rec[i][0], rec[i][1], rec[i][2], rec[i][3]);
    return 0;
}

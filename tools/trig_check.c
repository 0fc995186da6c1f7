/* Exhaustive check of pm_detmath.h's sin / cos over every float in
 * [-1, 8] (the renderer's angles lie in [-pi/4, 9 pi/4]): the float result
 * against libm's double sin / cos rounded to float. Prints the count of
 * results 1 ulp off and of results more than 1 ulp off (must be 0).
 *   gcc -O2 -fopenmp -ffp-contract=off tools/trig_check.c -lm -o /tmp/trig_check */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include "../include/pm_detmath.h"

static uint32_t fb(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }
static int64_t ulps(float a, float b) {
    int32_t ia = (int32_t)fb(a), ib = (int32_t)fb(b);
    if (ia < 0) ia = (int32_t)0x80000000 - ia;
    if (ib < 0) ib = (int32_t)0x80000000 - ib;
    int64_t d = (int64_t)ia - ib;
    return d < 0 ? -d : d;
}
int main(void) {
    long long one = 0, more = 0, n = 0;
    const float lo = -1.0f, hi = 8.0f;
    const uint32_t ulo = fb(lo) & 0x7fffffffu, uhi = fb(hi);
    /* negatives down to -1, then 0 .. 8 */
#pragma omp parallel for reduction(+ : one, more, n) schedule(dynamic, 1 << 16)
    for (int64_t i = -(int64_t)ulo; i <= (int64_t)uhi; ++i) {
        uint32_t u = i < 0 ? (uint32_t)(-i) | 0x80000000u : (uint32_t)i;
        float x;
        memcpy(&x, &u, 4);
        float s, c;
        pmdm_sincosf(x, &s, &c);
        const int64_t es = ulps(s, (float)sin((double)x)), ec = ulps(c, (float)cos((double)x));
        one += (es == 1) + (ec == 1);
        more += (es > 1) + (ec > 1);
        n += 2;
    }
    printf("values %lld: exact %lld, 1 ulp %lld, > 1 ulp %lld\n", n, n - one - more, one, more);
    return more != 0;
}

/*
 * pm_detmath.h — deterministic scalar math shared by the HIP kernels and the
 * CPU oracle (a tiny "libm" for this renderer, not part of either algorithm).
 *
 * Why it exists: the reference evaluates sinf/cosf/atan2f under
 * --use_fast_math (cuda_render/CMakeLists.txt:45-51), i.e. with
 * implementation-defined accuracy. To make GPU-vs-oracle parity BIT-EXACT
 * (photon positions, per-record photon counts) both sides evaluate the
 * transcendentals through the functions below, which use only IEEE-754
 * basic operations (+ - * / sqrt) in double precision and round once to
 * float. With -ffp-contract=off on both compilers (hipcc and gcc) every
 * result is identical on gfx950 and x86-64.
 *
 * Also holds the counter-based RNG that replaces the reference's cuRAND
 * MTGP32 stream (util/random/cudarandom.cpp:17-26, seed 777 at
 * util/random/cudarandom.h:15): Philox4x32-10 keyed on (seed, 0), counter =
 * (photon slot, pass, 0, 0). Same stream on both sides, no buffer.
 *
 * Accuracy: sin/cos/atan2 are within 1 ulp of the correctly rounded float
 * result (tests/test_oracle_kat.py checks them against libm in double).
 */
#ifndef PM_DETMATH_H
#define PM_DETMATH_H

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define PMDM_FN __host__ __device__ inline
#else
#define PMDM_FN static inline
#endif

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

/* pi/2 split into a 33-bit head (exact k*head for k < 2^20) and a tail. */
#define PMDM_PIO2_HI 1.57079632673412561417e+00
#define PMDM_PIO2_LO 6.07710050650619224932e-11
#define PMDM_TWO_OVER_PI 6.36619772367581382433e-01
#define PMDM_PI 3.14159265358979311600e+00
#define PMDM_PI_2 1.57079632679489655800e+00

/* sin and cos on |r| <= pi/4 + tiny: minimax polynomials for a float
 * result evaluated in double (|sin(r)/r - poly| < 2^-37.5, |cos(r) - poly| <
 * 2^-34.6 — the published coefficients of FreeBSD/musl __sindf / __cosdf),
 * so the one rounding to float is correct but for values within ~1e-11 of a
 * rounding midpoint: within 1 ulp everywhere. Round 5: these replace Taylor
 * series to r^19 / r^20 (~48 double operations per sincos -> ~26). */
PMDM_FN double pmdm_sin_kern(double r) {
    const double S1 = -0x15555554cbac77.0p-55, S2 = 0x111110896efbb2.0p-59;
    const double S3 = -0x1a00f9e2cae774.0p-65, S4 = 0x16cd878c3b46a7.0p-71;
    double z = r * r;
    double w = z * z;
    double q = S3 + z * S4;
    double s = z * r;
    return (r + s * (S1 + z * S2)) + (s * w) * q;
}

PMDM_FN double pmdm_cos_kern(double r) {
    const double C0 = -0x1ffffffd0c5e81.0p-54, C1 = 0x155553e1053a42.0p-57;
    const double C2 = -0x16c087e80f1e27.0p-62, C3 = 0x199342e0ee5069.0p-68;
    double z = r * r;
    double w = z * z;
    double q = C2 + z * C3;
    return ((1.0 + z * C0) + w * C1) + (w * z) * q;
}

/* Shared range reduction: x = k*pi/2 + r. Valid for |x| < 2^19 (all our
 * arguments are angles in [-2pi, 4pi]). */
PMDM_FN double pmdm_reduce(double x, int *quadrant) {
    double kf = x * PMDM_TWO_OVER_PI;
    /* round half away from zero; trunc == (double)(int64_t) here, one op on gfx950 */
    kf = (kf >= 0.0) ? __builtin_trunc(kf + 0.5) : -__builtin_trunc(0.5 - kf);
    *quadrant = (int)kf & 3;
    return (x - kf * PMDM_PIO2_HI) - kf * PMDM_PIO2_LO;
}

PMDM_FN float pmdm_sinf(float xf) {
    int q;
    double r = pmdm_reduce((double)xf, &q);
    double s = pmdm_sin_kern(r), c = pmdm_cos_kern(r);
    double v = (q == 0) ? s : (q == 1) ? c : (q == 2) ? -s : -c;
    return (float)v;
}

PMDM_FN float pmdm_cosf(float xf) {
    int q;
    double r = pmdm_reduce((double)xf, &q);
    double s = pmdm_sin_kern(r), c = pmdm_cos_kern(r);
    double v = (q == 0) ? c : (q == 1) ? -s : (q == 2) ? -c : s;
    return (float)v;
}

/* sin and cos of one angle with a single reduction; bit-identical to
 * pmdm_sinf / pmdm_cosf (same operations). */
PMDM_FN void pmdm_sincosf(float xf, float *sf, float *cf) {
    int q;
    double r = pmdm_reduce((double)xf, &q);
    double s = pmdm_sin_kern(r), c = pmdm_cos_kern(r);
    *sf = (float)((q == 0) ? s : (q == 1) ? c : (q == 2) ? -s : -c);
    *cf = (float)((q == 0) ? c : (q == 1) ? -s : (q == 2) ? -c : s);
}

/* atan on [0, tan(pi/16)]: odd Taylor series to t^27. */
PMDM_FN double pmdm_atan_small(double t) {
    double z = t * t;
    double p = 1.0 / 27.0;
    p = -p * z + 1.0 / 25.0;
    p = -p * z + 1.0 / 23.0;
    p = -p * z + 1.0 / 21.0;
    p = -p * z + 1.0 / 19.0;
    p = -p * z + 1.0 / 17.0;
    p = -p * z + 1.0 / 15.0;
    p = -p * z + 1.0 / 13.0;
    p = -p * z + 1.0 / 11.0;
    p = -p * z + 1.0 / 9.0;
    p = -p * z + 1.0 / 7.0;
    p = -p * z + 1.0 / 5.0;
    p = -p * z + 1.0 / 3.0;
    p = -p * z + 1.0;
    return t * p;
}

/* atan2f with C semantics for finite non-(0,0) inputs; (0,0) -> 0 or pi. */
PMDM_FN float pmdm_atan2f(float yf, float xf) {
    double y = (double)yf, x = (double)xf;
    double ax = x < 0.0 ? -x : x, ay = y < 0.0 ? -y : y;
    double r;
    if (ax == 0.0 && ay == 0.0) {
        r = 0.0;
    } else {
        int swap = ay > ax;
        double a = swap ? ax / ay : ay / ax; /* [0,1] */
        /* two argument halvings: atan(a) = 4 atan(t2) */
        double t = a / (1.0 + __builtin_sqrt(1.0 + a * a));
        t = t / (1.0 + __builtin_sqrt(1.0 + t * t));
        r = 4.0 * pmdm_atan_small(t);
        if (swap) r = PMDM_PI_2 - r;
    }
    if (x < 0.0) r = PMDM_PI - r;
    if (y < 0.0) r = -r;
    return (float)r;
}

/* ---------------------------------------------------------------------- */
/* Philox4x32-10 (Salmon et al., SC'11), key = (k0, k1), counter c[4].    */
/* ---------------------------------------------------------------------- */
PMDM_FN void pmdm_philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                uint32_t k0, uint32_t k1, uint32_t out[4]) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
    for (int i = 0; i < 10; ++i) {
        uint64_t p0 = (uint64_t)M0 * c0;
        uint64_t p1 = (uint64_t)M1 * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n1 = lo1;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        uint32_t n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += W0; k1 += W1;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* uint32 -> float in [0,1) with 24 random bits (exactly representable). */
PMDM_FN float pmdm_u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

#endif /* PM_DETMATH_H */

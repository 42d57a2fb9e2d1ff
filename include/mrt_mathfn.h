/* mrt_mathfn.h -- the transcendental functions of the render path's numerics contract.
 *
 * The reference calls glibc's sinf/cosf/tanf/logf/powf/atan2f/asinf (pcg.cpp:92-93, camera.h:22,
 * scene_object.cpp:36-37, volumes.cpp:24, material.h:109, sphere.cpp:7-8, texture.cpp:9).  This
 * project defines each as ONE deterministic evaluation in double precision followed by one
 * rounding to float.  Every operation below is a correctly rounded IEEE double add, sub, mul, div,
 * sqrt, rint or an explicit fma(), so the host (x86-64, -ffp-contract=off) and the device (gfx950,
 * hipcc -ffp-contract=off) produce the same bits.  The same functions are interposed into the exact
 * reference build (oracle/ref/harness.cpp, MRT_MATHMATCH) and used by the C restatement and the
 * host scene builder, so reference, oracle and GPU agree bit for bit by construction.
 * Accuracy before the final rounding is a few ulp of double, so the float results equal the
 * correctly rounded value except for ~1e-8 of arguments.
 */
#ifndef MRT_MATHFN_H
#define MRT_MATHFN_H

#if defined(__HIPCC__) || defined(__HIP__)
#define MRT_HD static __host__ __device__ inline
#else
#define MRT_HD static inline
#include <math.h>
#include <stdint.h>
#include <string.h>
#endif

/* Polynomial coefficients.  On the device each is materialised in an SGPR pair at its use (an
 * opaque move the compiler cannot hoist): double literals cannot be instruction operands on gfx9,
 * and hoisted out of the path loop they would pin ~30 VGPRs for the whole kernel.  The value is
 * the same double either way. */
#if defined(__HIP_DEVICE_COMPILE__)
__device__ static inline double mrt_dc_dev(double c) {
    unsigned long long b = __builtin_bit_cast(unsigned long long, c);
    unsigned int lo = (unsigned int)b, hi = (unsigned int)(b >> 32);
    asm volatile("" : "+s"(lo), "+s"(hi));
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
#define MRT_DC(x) mrt_dc_dev(x)
#else
#define MRT_DC(x) (x)
#endif

/* ---- sin / cos: Cody-Waite reduction by pi/2 (|x| < 2^20), Taylor kernels on [-pi/4, pi/4] ---- */
MRT_HD void mrt_sincos_d(double x, double* s, double* c) {
    const double two_over_pi = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;  /* first 33 bits of pi/2 */
    const double pio2_1t = 6.07710050650619224932e-11; /* pi/2 - pio2_1 */
    double k = rint(x * MRT_DC(two_over_pi));
    double r = fma(-k, MRT_DC(pio2_1), x);
    r = fma(-k, MRT_DC(pio2_1t), r);
    double z = r * r;
    /* sin r = r + r^3 P(z) */
    double p = MRT_DC(2.8114572543455206e-15);   /*  1/17! */
    p = fma(p, z, MRT_DC(-7.6471637318198164e-13)); /* -1/15! */
    p = fma(p, z, MRT_DC(1.6059043836821613e-10));  /*  1/13! */
    p = fma(p, z, MRT_DC(-2.5052108385441720e-08)); /* -1/11! */
    p = fma(p, z, MRT_DC(2.7557319223985893e-06));  /*  1/9!  */
    p = fma(p, z, MRT_DC(-1.9841269841269841e-04)); /* -1/7!  */
    p = fma(p, z, MRT_DC(8.3333333333333332e-03));  /*  1/5!  */
    p = fma(p, z, MRT_DC(-1.6666666666666666e-01)); /* -1/3!  */
    double sr = fma(p * z, r, r);
    /* cos r = (1 - z/2) + z^2 Q(z) */
    double q = MRT_DC(-1.5619206968586225e-16);  /* -1/18! */
    q = fma(q, z, MRT_DC(4.7794773323873853e-14));  /*  1/16! */
    q = fma(q, z, MRT_DC(-1.1470745597729725e-11)); /* -1/14! */
    q = fma(q, z, MRT_DC(2.0876756987868099e-09));  /*  1/12! */
    q = fma(q, z, MRT_DC(-2.7557319223985888e-07)); /* -1/10! */
    q = fma(q, z, MRT_DC(2.4801587301587302e-05));  /*  1/8!  */
    q = fma(q, z, MRT_DC(-1.3888888888888889e-03)); /* -1/6!  */
    q = fma(q, z, MRT_DC(4.1666666666666664e-02));  /*  1/4!  */
    double cr = fma(q * z, z, fma(-0.5, z, 1.0));
    long long n = (long long)k & 3;
    double ss = (n & 1) ? cr : sr;
    double cc = (n & 1) ? sr : cr;
    *s = (n & 2) ? -ss : ss;
    *c = ((n + 1) & 2) ? -cc : cc;
}
MRT_HD float mrt_sinf(float x) {
    double s, c;
    mrt_sincos_d((double)x, &s, &c);
    return (float)s;
}
MRT_HD float mrt_cosf(float x) {
    double s, c;
    mrt_sincos_d((double)x, &s, &c);
    return (float)c;
}
MRT_HD float mrt_tanf(float x) {
    double s, c;
    mrt_sincos_d((double)x, &s, &c);
    return (float)(s / c);
}

/* ---- log: x = m 2^e, m in [sqrt(1/2), sqrt(2)), log m = 2 atanh((m-1)/(m+1)) ---- */
MRT_HD double mrt_log_d(double x) {
    if (!(x > 0.0)) return x == 0.0 ? -1.0 / 0.0 : (x - x) / (x - x); /* log 0 = -inf, log(<0 or NaN) = NaN */
    if (x == 1.0 / 0.0) return x;
    int e = 0;
    if (x < 2.2250738585072014e-308) { /* subnormal */
        x *= 18014398509481984.0;     /* 2^54 */
        e = -54;
    }
    uint64_t b;
    memcpy(&b, &x, 8);
    e += (int)((b >> 52) & 0x7FF) - 1023;
    b = (b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull;
    double m;
    memcpy(&m, &b, 8);
    if (m > 1.4142135623730951) {
        m *= 0.5;
        e += 1;
    }
    double s = (m - 1.0) / (m + 1.0);
    double z = s * s;
    double p = MRT_DC(2.0 / 23.0);
    p = fma(p, z, MRT_DC(2.0 / 21.0));
    p = fma(p, z, MRT_DC(2.0 / 19.0));
    p = fma(p, z, MRT_DC(2.0 / 17.0));
    p = fma(p, z, MRT_DC(2.0 / 15.0));
    p = fma(p, z, MRT_DC(2.0 / 13.0));
    p = fma(p, z, MRT_DC(2.0 / 11.0));
    p = fma(p, z, MRT_DC(2.0 / 9.0));
    p = fma(p, z, MRT_DC(2.0 / 7.0));
    p = fma(p, z, MRT_DC(2.0 / 5.0));
    p = fma(p, z, MRT_DC(2.0 / 3.0));
    double lm = fma(s * z, p, 2.0 * s);
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    double de = (double)e;
    return fma(de, MRT_DC(ln2_hi), fma(de, MRT_DC(ln2_lo), lm));
}
MRT_HD float mrt_logf(float x) { return (float)mrt_log_d((double)x); }

/* ---- pow: the render path only raises to the 5th power (fresnel_schlick, material.h:109) ---- */
MRT_HD float mrt_pow5f(float x) {
    double d = (double)x;
    double d2 = d * d; /* exact: 48 significant bits */
    return (float)((d2 * d2) * d);
}

/* ---- atan / atan2 / asin (sphere uv, sphere.cpp:6-11) ---- */
MRT_HD double mrt_atan_d(double x) { /* |x| <= 1 */
    /* two half-angle steps: atan x = 2 atan(x / (1 + sqrt(1 + x^2))) -> |t| <= tan(pi/16) */
    double t = x / (1.0 + sqrt(fma(x, x, 1.0)));
    t = t / (1.0 + sqrt(fma(t, t, 1.0)));
    double z = t * t;
    double p = MRT_DC(-1.0 / 27.0);
    p = fma(p, z, MRT_DC(1.0 / 25.0));
    p = fma(p, z, MRT_DC(-1.0 / 23.0));
    p = fma(p, z, MRT_DC(1.0 / 21.0));
    p = fma(p, z, MRT_DC(-1.0 / 19.0));
    p = fma(p, z, MRT_DC(1.0 / 17.0));
    p = fma(p, z, MRT_DC(-1.0 / 15.0));
    p = fma(p, z, MRT_DC(1.0 / 13.0));
    p = fma(p, z, MRT_DC(-1.0 / 11.0));
    p = fma(p, z, MRT_DC(1.0 / 9.0));
    p = fma(p, z, MRT_DC(-1.0 / 7.0));
    p = fma(p, z, MRT_DC(1.0 / 5.0));
    p = fma(p, z, MRT_DC(-1.0 / 3.0));
    return 4.0 * fma(t * z, p, t);
}
MRT_HD double mrt_atan2_d(double y, double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    /* the two constants made by the instructions themselves where used, not hoisted into register
       pairs held across the caller's loops (book2's path kernel spilled them to scratch) */
    int pl, ph, ql, qh;
    __asm__ volatile("v_mov_b32 %0, 0x54442d18\n\tv_mov_b32 %1, 0x400921fb\n\tv_mov_b32 %2, 0x54442d18\n\tv_mov_b32 %3, 0x3ff921fb"
                     : "=v"(pl), "=v"(ph), "=v"(ql), "=v"(qh));
    const double pi = __builtin_bit_cast(double, ((unsigned long long)(unsigned)ph << 32) | (unsigned)pl);
    const double pio2 = __builtin_bit_cast(double, ((unsigned long long)(unsigned)qh << 32) | (unsigned)ql);
#else
    const double pi = 3.14159265358979311600e+00, pio2 = 1.57079632679489655800e+00;
#endif
    if (x != x || y != y) return x + y;
    if (y == 0.0) {
        if (x > 0.0 || (x == 0.0 && !signbit(x))) return y;   /* +-0 */
        return signbit(y) ? -pi : pi;
    }
    if (x == 0.0) return y > 0.0 ? pio2 : -pio2;
    double ax = fabs(x), ay = fabs(y), r;
    if (ax == 1.0 / 0.0 || ay == 1.0 / 0.0) {
        double a = ay == 1.0 / 0.0 ? (ax == 1.0 / 0.0 ? pio2 * 0.5 : pio2) : 0.0;
        r = a;
    } else if (ay <= ax) {
        r = mrt_atan_d(ay / ax);
    } else {
        r = pio2 - mrt_atan_d(ax / ay);
    }
    if (x < 0.0) r = pi - r;
    return y < 0.0 ? -r : r;
}
MRT_HD float mrt_atan2f(float y, float x) { return (float)mrt_atan2_d((double)y, (double)x); }
MRT_HD float mrt_asinf(float x) {
    double d = (double)x;
    if (!(fabs(d) <= 1.0)) return (float)((d - d) / (d - d)); /* NaN */
    return (float)mrt_atan2_d(d, sqrt((1.0 - d) * (1.0 + d)));
}

/* ---- log10 / exp / pow: the Drago tone map of the image output (main.cpp:421-439) ---- */
MRT_HD float mrt_log10f(float x) {
    const double inv_ln10 = 4.34294481903251816668e-01; /* 1 / ln 10 */
    return (float)(mrt_log_d((double)x) * MRT_DC(inv_ln10));
}
/* e^x: x = k ln2 + r, |r| <= ln2/2, Taylor to r^14, scaled by 2^k through the exponent field */
MRT_HD double mrt_exp_d(double x) {
    if (x != x) return x;
    if (x > 709.0) return 1.0 / 0.0;
    if (x < -745.0) return 0.0;
    const double inv_ln2 = 1.44269504088896338700e+00;
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    double k = rint(x * MRT_DC(inv_ln2));
    double r = fma(-k, MRT_DC(ln2_hi), x);
    r = fma(-k, MRT_DC(ln2_lo), r);
    double p = MRT_DC(1.0 / 87178291200.0);       /* 1/14! */
    p = fma(p, r, MRT_DC(1.0 / 6227020800.0));    /* 1/13! */
    p = fma(p, r, MRT_DC(1.0 / 479001600.0));     /* 1/12! */
    p = fma(p, r, MRT_DC(1.0 / 39916800.0));      /* 1/11! */
    p = fma(p, r, MRT_DC(1.0 / 3628800.0));       /* 1/10! */
    p = fma(p, r, MRT_DC(1.0 / 362880.0));        /* 1/9!  */
    p = fma(p, r, MRT_DC(1.0 / 40320.0));         /* 1/8!  */
    p = fma(p, r, MRT_DC(1.0 / 5040.0));          /* 1/7!  */
    p = fma(p, r, MRT_DC(1.0 / 720.0));           /* 1/6!  */
    p = fma(p, r, MRT_DC(1.0 / 120.0));           /* 1/5!  */
    p = fma(p, r, MRT_DC(1.0 / 24.0));            /* 1/4!  */
    p = fma(p, r, MRT_DC(1.0 / 6.0));             /* 1/3!  */
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    double e = fma(p, r, 1.0);
    /* e * 2^k in two exact steps (k in [-1075, 1024]) */
    int ki = (int)k;
    int k1 = ki / 2, k2 = ki - k1;
    uint64_t b1 = (uint64_t)(k1 + 1023) << 52, b2 = (uint64_t)(k2 + 1023) << 52;
    double s1, s2;
    memcpy(&s1, &b1, 8);
    memcpy(&s2, &b2, 8);
    return (e * s1) * s2;
}
MRT_HD float mrt_expf(float x) { return (float)mrt_exp_d((double)x); }
/* x^y for the tone map's x in [0, 1], y > 0 (and the general finite case x > 0) */
MRT_HD float mrt_powf(float x, float y) {
    if (y == 5.0f) return mrt_pow5f(x);
    if (x == 1.0f || y == 0.0f) return 1.0f;
    if (x == 0.0f) return y > 0.0f ? 0.0f : 1.0f / 0.0f;
    if (!(x > 0.0f)) return (x - x) / (x - x); /* negative base with non-integer y, or NaN */
    return (float)mrt_exp_d((double)y * mrt_log_d((double)x));
}

#endif

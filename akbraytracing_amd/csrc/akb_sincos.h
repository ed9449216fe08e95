// Correctly rounded sin / cos of one double, for the device-side tilt matrices (and a host build
// of the same code for its CPU test).
//
// The reference forms R_y, R_z of rotate_vectors (AKB_raytrace_20250312.py:917-927) with numpy's
// cos / sin of the tilt angles; building them on the device removes a host round trip from every
// ray_wave run. The value is evaluated in double-double (Taylor series of sin and cos to 16
// terms at most, ~2^-100 relative) and rounded once, so it is the correctly rounded result except in the
// vanishingly rare case of an argument within ~2^-100 of a rounding boundary. glibc's sin / cos,
// which numpy calls for float64, are not correctly rounded: measured here they differ from the
// correctly rounded value on ~0.13 % of random arguments (by one ulp), so a matrix entry can sit
// one ulp from numpy's. That is inside the tilt stage's tolerance, which is already set by the
// per-ray arctan feeding the tilt angle.
//
// |x| <= pi/4 needs no reduction (tilt angles are milliradians; small |x| needs few terms).
// Larger |x| is reduced by x - k pi/2 with a three-part pi/2 in double-double (faithful, correctly rounded unless x sits
// near a multiple of pi/2); |x| >= 2^20 and non-finite x fall back to the library sin / cos.
#pragma once

#include <math.h>

#if defined(__HIPCC__)
#define AKB_SC_FN __host__ __device__ __forceinline__
#else
#define AKB_SC_FN static inline
#endif

namespace akb_sc {

struct DD {
    double hi, lo;
};

AKB_SC_FN DD two_sum(double a, double b) {
    const double s = a + b;
    const double bb = s - a;
    return DD{s, (a - (s - bb)) + (b - bb)};
}
AKB_SC_FN DD fast_two_sum(double a, double b) {
    const double s = a + b;
    return DD{s, b - (s - a)};
}
AKB_SC_FN DD two_prod(double a, double b) {
    const double p = a * b;
    return DD{p, __builtin_fma(a, b, -p)};
}
AKB_SC_FN DD dd_add(DD a, DD b) {
    DD s = two_sum(a.hi, b.hi);
    const DD t = two_sum(a.lo, b.lo);
    s.lo = s.lo + t.hi;
    s = fast_two_sum(s.hi, s.lo);
    s.lo = s.lo + t.lo;
    return fast_two_sum(s.hi, s.lo);
}
AKB_SC_FN DD dd_mul(DD a, DD b) {
    DD p = two_prod(a.hi, b.hi);
    p.lo = p.lo + (a.hi * b.lo + a.lo * b.hi);
    return fast_two_sum(p.hi, p.lo);
}

// (-1)^k / (2k+1)! and (-1)^k / (2k)!, k = 0..15, as double-double (hi, lo)
#define AKB_SC_SIN_TABLE                                                                           \
    {{0x1.0000000000000p+0, 0x0.0p+0},                                                             \
     {-0x1.5555555555555p-3, -0x1.5555555555555p-57},                                              \
     {0x1.1111111111111p-7, 0x1.1111111111111p-63},                                                \
     {-0x1.a01a01a01a01ap-13, -0x1.a01a01a01a01ap-73},                                             \
     {0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73},                                              \
     {-0x1.ae64567f544e4p-26, 0x1.c062e06d1f209p-80},                                              \
     {0x1.6124613a86d09p-33, 0x1.f28e0cc748ebep-87},                                               \
     {-0x1.ae7f3e733b81fp-41, -0x1.1d8656b0ee8cbp-97},                                             \
     {0x1.952c77030ad4ap-49, 0x1.ac981465ddc6cp-103},                                              \
     {-0x1.2f49b46814157p-57, -0x1.2650f61dbdcb4p-112},                                            \
     {0x1.71b8ef6dcf572p-66, -0x1.d043ae40c4647p-120},                                             \
     {-0x1.761b41316381ap-75, 0x1.3423c7d91404fp-130},                                             \
     {0x1.3f3ccdd165fa9p-84, -0x1.58ddadf344487p-139},                                             \
     {-0x1.d1ab1c2dccea3p-94, -0x1.054d0c78aea14p-149},                                            \
     {0x1.259f98b4358adp-103, 0x1.eaf8c39dd9bc5p-157},                                             \
     {-0x1.434d2e783f5bcp-113, -0x1.0b87b91be9affp-167}}
#define AKB_SC_COS_TABLE                                                                           \
    {{0x1.0000000000000p+0, 0x0.0p+0},                                                             \
     {-0x1.0000000000000p-1, 0x0.0p+0},                                                            \
     {0x1.5555555555555p-5, 0x1.5555555555555p-59},                                                \
     {-0x1.6c16c16c16c17p-10, 0x1.f49f49f49f49fp-65},                                              \
     {0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76},                                               \
     {-0x1.27e4fb7789f5cp-22, -0x1.cbbc05b4fa99ap-76},                                             \
     {0x1.1eed8eff8d898p-29, -0x1.2aec959e14c06p-83},                                              \
     {-0x1.93974a8c07c9dp-37, -0x1.05d6f8a2efd1fp-92},                                             \
     {0x1.ae7f3e733b81fp-45, 0x1.1d8656b0ee8cbp-101},                                              \
     {-0x1.6827863b97d97p-53, -0x1.eec01221a8b0bp-107},                                            \
     {0x1.e542ba4020225p-62, 0x1.ea72b4afe3c2fp-120},                                              \
     {-0x1.0ce396db7f853p-70, 0x1.aebcdbd20331cp-124},                                             \
     {0x1.f2cf01972f578p-80, -0x1.9ada5fcc1ab14p-135},                                             \
     {-0x1.88e85fc6a4e5ap-89, 0x1.71c37ebd16540p-143},                                             \
     {0x1.0a18a2635085dp-98, 0x1.b9e2e28e1aa54p-153},                                              \
     {-0x1.3932c5047d60ep-108, -0x1.832b7b530a627p-162}}

// sum_{k <= top} c[k] z^k by Horner in double-double
AKB_SC_FN DD series(const double (&c)[16][2], DD z, int top) {
    DD p{c[top][0], c[top][1]};
    for (int k = top - 1; k >= 0; --k) p = dd_add(dd_mul(p, z), DD{c[k][0], c[k][1]});
    return p;
}

// highest Taylor index needed for |r| <= pi/4 * 2^-e: the first omitted term of either series
// stays below 2^-112 of the result (one index of margin on top)
AKB_SC_FN int series_top(double ar) {
    if (ar < 0x1p-21) return 3;
    if (ar < 0x1p-13) return 4;
    if (ar < 0x1p-11) return 5;
    if (ar < 0x1p-9) return 6;
    if (ar < 0x1p-7) return 7;
    if (ar < 0x1p-5) return 8;
    if (ar < 0x1p-4) return 9;
    if (ar < 0x1p-3) return 11;
    if (ar < 0x1p-2) return 13;
    return 15;
}

// sin(x) (want_cos false) or cos(x), rounded to nearest
AKB_SC_FN double sin_cos_cr(double x, bool want_cos) {
    const double ax = fabs(x);
    if (!(ax < 0x1p20)) return want_cos ? cos(x) : sin(x);  // huge or non-finite: library
    if (ax < 0x1p-27) return want_cos ? 1.0 : x;  // to within half an ulp (keeps -0)
    DD r{x, 0.0};
    long long q = 0;
    if (ax > 0x1.921fb54442d18p-1) {  // pi/4
        const double k = rint(x * 0x1.45f306dc9c883p-1);  // x * 2/pi
        q = (long long)k;
        const DD p0 = two_prod(k, 0x1.921fb54442d18p+0);
        const DD p1 = two_prod(k, 0x1.1a62633145c07p-54);
        r = dd_add(r, DD{-p0.hi, -p0.lo});
        r = dd_add(r, DD{-p1.hi, -p1.lo});
        r = dd_add(r, DD{-(k * -0x1.f1976b7ed8fbcp-110), 0.0});
    }
    // quadrant: sin -> (S, C, -S, -C), cos -> (C, -S, -C, S) for q mod 4 = 0..3
    const int qq = (int)(q & 3);
    const bool use_cos = want_cos ? (qq == 0 || qq == 2) : (qq == 1 || qq == 3);
    const bool negate = want_cos ? (qq == 1 || qq == 2) : (qq == 2 || qq == 3);
    const DD z = dd_mul(r, r);
    const int top = series_top(fabs(r.hi));
    double v;
    if (use_cos) {
        const double kCos[16][2] = AKB_SC_COS_TABLE;
        v = series(kCos, z, top).hi;
    } else {
        const double kSin[16][2] = AKB_SC_SIN_TABLE;
        v = dd_mul(r, series(kSin, z, top)).hi;
    }
    return negate ? -v : v;
}

AKB_SC_FN void sincos_cr(double x, double* s, double* c) {
    *s = sin_cos_cr(x, false);
    *c = sin_cos_cr(x, true);
}

}  // namespace akb_sc

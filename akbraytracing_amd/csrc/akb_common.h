// Shared helpers of the gfx950 kernels behind include/akb_raytrace.h.
//
// Every translation unit is compiled with -ffp-contract=off: the trace kernels reproduce numpy's
// evaluation order operation by operation (each product and sum rounded on its own), which is
// what makes them bit-identical to the reference's numpy expressions. Where an FMA is wanted
// (Huygens complex accumulation, tolerance-checked) it is written explicitly.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string>

#include "../../include/akb_raytrace.h"

// Wave priority of the latency-bound kernels (the faithful chain's, the trace's sums and tilt
// parameters, the PSF): in a pipelined step they run on the critical path while the trace passes'
// FP64-bound waves share their SIMDs, so each of their waves issues first (s_setprio); the passes,
// throughput work with slack in the step, take the remaining issue slots.
#ifndef AKB_NO_CHAIN_PRIO
#define AKB_CHAIN_PRIORITY() __builtin_amdgcn_s_setprio(3)
#else
#define AKB_CHAIN_PRIORITY() ((void)0)
#endif

namespace akb {

// thread-local last error, surfaced by akb_last_error()
void set_error(const char* fmt, ...);
void clear_error();

#define AKB_HIP_CHECK(expr)                                                                  \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess) {                                                              \
            ::akb::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                             __LINE__);                                                      \
            return AKB_E_HIP;                                                                \
        }                                                                                    \
    } while (0)

#define AKB_REQUIRE(cond, msg)                                                    \
    do {                                                                          \
        if (!(cond)) {                                                            \
            ::akb::set_error("invalid argument: %s (%s)", msg, #cond);            \
            return AKB_E_INVALID;                                                 \
        }                                                                         \
    } while (0)

// check the launch that was just issued
inline int launch_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("launch of %s failed: %s", what, hipGetErrorString(e));
        return AKB_E_HIP;
    }
    return AKB_OK;
}

constexpr int kBlock = 256;  // 4 waves of 64

// Grid for a grid-stride elementwise kernel: enough workgroups to fill 256 CUs several times
// over, capped so each thread still loops a few times on very large arrays. Streaming kernels
// that mix several read and write rows reach more of HBM with larger grids (measured on MI355X:
// 7 reads + 4 writes per element, 4.6 TB/s at 2k workgroups, 5.1 TB/s at 16k), so they pass a
// larger cap.
inline unsigned grid_for(int64_t n, int per_thread_min = 1, int64_t cap = 256 * 16) {
    int64_t blocks = (n + (int64_t)kBlock * per_thread_min - 1) / ((int64_t)kBlock * per_thread_min);
    if (blocks < 1) blocks = 1;
    return (unsigned)(blocks > cap ? cap : blocks);
}
constexpr int64_t kStreamGridCap = 256 * 64;

// 3-vector view of a (3, ld) SoA block with element increment inc (0 = broadcast)
struct V3In {
    const double* p;
    int64_t ld;
    int64_t inc;
    __device__ __forceinline__ double x(int64_t i) const { return p[i * inc]; }
    __device__ __forceinline__ double y(int64_t i) const { return p[ld + i * inc]; }
    __device__ __forceinline__ double z(int64_t i) const { return p[2 * ld + i * inc]; }
};
#ifndef AKB_STAGE_NT
#define AKB_STAGE_NT 1  // the stage kernels' row stores nontemporal (norm_vector / normalize_vector 0.70 -> 0.82 of HBM; 0 for A/B)
#endif
struct V3Out {
    double* p;
    int64_t ld;
    __device__ __forceinline__ void store(int64_t i, double x, double y, double z) const {
        if (AKB_STAGE_NT) {
            __builtin_nontemporal_store(x, p + i);
            __builtin_nontemporal_store(y, p + ld + i);
            __builtin_nontemporal_store(z, p + 2 * ld + i);
        } else {
            p[i] = x;
            p[ld + i] = y;
            p[2 * ld + i] = z;
        }
    }
};

// base[off / 8] for a byte offset that fits 32 bits: the access takes a scalar (wave-uniform) base
// plus a 32-bit lane offset (global_load / global_store saddr form) instead of a per-lane 64-bit
// address formed with 64-bit vector adds
__device__ __forceinline__ double ld_off(const double* base, uint32_t off) {
    return *(const double*)((const char*)base + off);
}
__device__ __forceinline__ void st_off(double* base, uint32_t off, double v) { *(double*)((char*)base + off) = v; }

struct Quadric {
    double a, b, c, d, e, f, g, h, i, j;
};

inline Quadric quadric_from(const double* c) {
    return Quadric{c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], c[8], c[9]};
}

// ---- per-ray arithmetic, each in the reference's numpy association order ----

// x / s for several x sharing one s, each correctly rounded: inv = RN(1/s) (an IEEE division),
// q = RN(x * inv), then one FMA correction q + (x - s q) inv, which is RN(x/s) whenever no
// overflow or underflow occurs (Markstein 1990; 5.4e8 adversarial cases checked against x / s).
// The r == 0 test returns q unchanged when it is already exact, which also keeps the sign of a
// zero quotient (x = -0). Zero or non-finite s is caught by the callers' zero-norm flags.
__device__ __forceinline__ double div_shared(double x, double s, double inv) {
    const double q = x * inv;
    const double r = __builtin_fma(-s, q, x);
    return r == 0.0 ? q : __builtin_fma(r, inv, q);
}

// The in-range cores of sqrt_cr and norm3_inv below (no range test of their own).
__device__ __forceinline__ double sqrt_core(double x) {
    const double r = __builtin_amdgcn_rsq(x);
    double g = x * r;
    double h = r * 0.5;
    const double e = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, e, g);
    const double d = __builtin_fma(-g, g, x);
    h = __builtin_fma(h, e, h);
    g = __builtin_fma(d, h, g);
    const double d2 = __builtin_fma(-g, g, x);
    return __builtin_fma(d2, h, g);
}
__device__ __forceinline__ double rcp_core(double s) {
    double y0 = __builtin_amdgcn_rcp(s);
    double e0 = __builtin_fma(-s, y0, 1.0);
    y0 = __builtin_fma(y0, e0, y0);
    e0 = __builtin_fma(-s, y0, 1.0);
    y0 = __builtin_fma(y0, e0, y0);
    const double r1 = __builtin_fma(-s, y0, 1.0);  // q = 1 * y0 = y0
    return __builtin_fma(r1, y0, y0);
}
__device__ __forceinline__ bool in_fast_range(double v) { return v >= 0x1p-767 && v <= 0x1p+1000; }

// x / d as hipcc's IEEE division computes it, without its operand scaling: hipcc emits
// v_div_scale (both operands), rcp + two Newton steps, the quotient and its residual, v_div_fmas
// and v_div_fixup. For |x| and |d| in [2^-300, 2^300] the scaling is the identity (exponent
// difference < 768, no operand, reciprocal or quotient near the denormals, numerator exponent
// far above 53), v_div_fmas is a plain FMA and v_div_fixup returns its input, so the core below
// gives the same bits in 8 instead of 12 instructions (checked bitwise by k_selftest).
__device__ __forceinline__ bool in_div_range(double v) {
    const double a = fabs(v);
    return a >= 0x1p-300 && a <= 0x1p+300;
}
__device__ __forceinline__ double div_core(double x, double d) {
    double y = __builtin_amdgcn_rcp(d);
    double e = __builtin_fma(-d, y, 1.0);
    y = __builtin_fma(y, e, y);
    e = __builtin_fma(-d, y, 1.0);
    y = __builtin_fma(y, e, y);
    const double q = x * y;
    const double r = __builtin_fma(-d, q, x);
    return __builtin_fma(r, y, q);
}
// every lane takes the core; a wave holding a lane outside the range (a uniform branch) computes
// the library quotient and selects it for those lanes
__device__ __forceinline__ double div_w(double x, double d) {
    const bool in = in_div_range(x) && in_div_range(d);
    double q = div_core(x, d);
    if (__builtin_expect(__ballot(!in) != 0, 0)) {
        const double ql = x / d;
        q = in ? q : ql;
    }
    return q;
}

// Correctly rounded square root without the tiny-input rescaling. hipcc's sqrt(double) on gfx950
// scales inputs below 2^-767 by 2^256 (cmp, cndmask, ldexp in; cndmask, ldexp out; class test for
// 0 / inf) around an rsq + Goldschmidt/Newton core. For inputs in [2^-767, 2^1000] the rescale is
// the identity and the special cases cannot occur, so the core alone - the same instruction
// sequence - gives the bit-identical result in fewer instructions. Everything else (zero,
// negatives, NaN, inf, tiny or huge values: never produced by the trace's unit-vector norms,
// discriminants and metre-scale segment lengths) takes sqrt() itself.
// The range test is wave-wide: every lane takes the core and only a wave holding a lane outside
// the range (a uniform branch) runs the library sqrt and selects it for those lanes - a per-lane
// branch would be if-converted into the library's scaling selects on every lane.
__device__ __forceinline__ double sqrt_cr(double x) {
    const bool in = in_fast_range(x);
    const double r = __builtin_amdgcn_rsq(x);
    double g = x * r;
    double h = r * 0.5;
    const double e = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, e, g);
    const double d = __builtin_fma(-g, g, x);
    h = __builtin_fma(h, e, h);
    g = __builtin_fma(d, h, g);
    const double d2 = __builtin_fma(-g, g, x);
    double s = __builtin_fma(d2, h, g);
    if (__builtin_expect(__ballot(!in) != 0, 0)) {
        const double sl = sqrt(x);
        s = in ? s : sl;
    }
    return s;
}

// np.linalg.norm(v, axis=0) for one column: sqrt((x*x + y*y) + z*z)
__device__ __forceinline__ double norm3(double x, double y, double z) {
    return sqrt_cr(x * x + y * y + z * z);
}

// div_shared for a divisor known to be positive (a norm): the residual is formed with the opposite
// sign, rn = RN(s q - x) = -RN(x - s q), so q - rn inv equals the corrected quotient for every
// non-zero residual and, for a zero residual, keeps q together with the sign of a zero quotient
// (x = +-0 gives rn = +0 and q - (+0) inv = q) without div_shared's compare and selects.
// s < 0 would lose the sign of a +0 quotient: the callers' divisors are norms.
__device__ __forceinline__ double div_pos(double x, double s, double inv) {
    const double q = x * inv;
    const double rn = __builtin_fma(s, q, -x);
    return __builtin_fma(-rn, inv, q);
}

// s = np.linalg.norm of (x, y, z) and inv = RN(1 / s), sharing sqrt_cr's range test: for a squared
// norm in [2^-767, 2^1000], s lies in [2^-384, 2^500], where hipcc's IEEE division 1 / s neither
// scales its operands (v_div_scale) nor fixes its result up (v_div_fmas / v_div_fixup are the
// identity), so the remaining rcp + two Newton steps + the final correction give its bits exactly
// in 7 instead of 11 instructions. Outside the range both take the library operations.
__device__ __forceinline__ void norm3_inv(double x, double y, double z, double& s, double& inv) {
    const double v = x * x + y * y + z * z;
    if (__builtin_expect(v >= 0x1p-767 && v <= 0x1p+1000, 1)) {
        const double r = __builtin_amdgcn_rsq(v);
        double g = v * r;
        double h = r * 0.5;
        const double e = __builtin_fma(-h, g, 0.5);
        g = __builtin_fma(g, e, g);
        const double d = __builtin_fma(-g, g, v);
        h = __builtin_fma(h, e, h);
        g = __builtin_fma(d, h, g);
        const double d2 = __builtin_fma(-g, g, v);
        s = __builtin_fma(d2, h, g);
        double y0 = __builtin_amdgcn_rcp(s);
        double e0 = __builtin_fma(-s, y0, 1.0);
        y0 = __builtin_fma(y0, e0, y0);
        e0 = __builtin_fma(-s, y0, 1.0);
        y0 = __builtin_fma(y0, e0, y0);
        const double r1 = __builtin_fma(-s, y0, 1.0);  // q = 1 * y0 = y0
        inv = __builtin_fma(r1, y0, y0);
    } else {
        s = sqrt(v);
        inv = 1.0 / s;
    }
}

// norm3_inv for a vector whose squared norm is ~1 or NaN: a reflection r = l - 2 (l.n) n of a unit
// direction l about a unit normal n has |r| = |l| = 1 up to rounding, so v = |r|^2 lies far inside
// norm3_inv's range and its range test (two compares and the exec-mask juggling around the
// library fallback) can go. v == 0 cannot occur for unit l and n, and if it does (it is returned
// in `zero` for the caller's flag, where s and inv are NaN) the flag sends the ray to the staged
// path, which applies the reference's value rule. A NaN input gives NaN as the checked form does.
__device__ __forceinline__ void norm3_inv_unit(double x, double y, double z, double& s, double& inv, bool& zero) {
    const double v = x * x + y * y + z * z;
    zero = v == 0.0;
    const double r = __builtin_amdgcn_rsq(v);
    double g = v * r;
    double h = r * 0.5;
    const double e = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, e, g);
    const double d = __builtin_fma(-g, g, v);
    h = __builtin_fma(h, e, h);
    g = __builtin_fma(d, h, g);
    const double d2 = __builtin_fma(-g, g, v);
    s = __builtin_fma(d2, h, g);
    double y0 = __builtin_amdgcn_rcp(s);
    double e0 = __builtin_fma(-s, y0, 1.0);
    y0 = __builtin_fma(y0, e0, y0);
    e0 = __builtin_fma(-s, y0, 1.0);
    y0 = __builtin_fma(y0, e0, y0);
    const double r1 = __builtin_fma(-s, y0, 1.0);
    inv = __builtin_fma(r1, y0, y0);
}

// np.arctan of an exit-ray slope (AKB_raytrace_20250312.py:2856-2857, :3583-3584). The slopes of a
// focusing system are small (|x| ~ 1e-5 for the reference AKB), where the Taylor series
// x - x^3/3 + ... + x^13/13 is exact to 2^-59 relative for |x| <= 2^-4 and x + (x z) P(z) rounds
// to within 0.51 ulp: 8 instructions instead of OCML's range-reduced rational (~45, including an
// IEEE division). Larger slopes take OCML's atan. Neither equals numpy's (glibc or its AVX-512
// SIMD routine) bit for bit; the tilt stage's tolerance covers it.
// OCML's atan out of line: its rational's constants then live only inside the call instead of
// occupying registers across the whole trace loop
__device__ __attribute__((noinline)) static double atan_lib(double x) { return atan(x); }

// fma(a, b, c) as one VOP3 v_fma_f64 with every operand in a VGPR: for a loop-invariant c (a
// polynomial coefficient) the compiler otherwise picks the two-address v_fmac_f64 and copies c into
// the destination first, one v_mov_b64 per term
__device__ __forceinline__ double fma3(double a, double b, double c) {
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__device__ __forceinline__ double atan_slope(double x) {
    if (__builtin_expect(fabs(x) <= 0x1p-4, 1)) {
        const double z = x * x;
        double P = 1.0 / 13.0;
        P = fma3(z, P, -1.0 / 11.0);
        P = fma3(z, P, 1.0 / 9.0);
        P = fma3(z, P, -1.0 / 7.0);
        P = fma3(z, P, 1.0 / 5.0);
        P = fma3(z, P, -1.0 / 3.0);
        return __builtin_fma(x * z, P, x);
    }
    return atan_lib(x);
}

// mirr_ray_intersection (EllipseRaytrace3D.py:23-43). Returns false when D <= 0 or NaN.
__device__ __forceinline__ bool quadric_hit(const Quadric& Q, double l, double m, double n, double p,
                                            double q, double r, bool negative, double& x, double& y,
                                            double& z) {
    const double A = Q.a * (l * l) + Q.b * (m * m) + Q.c * (n * n) + Q.d * m * l + Q.e * n * l +
                     Q.f * m * n;
    const double B = 2.0 * Q.a * p * l + 2.0 * Q.b * q * m + 2.0 * Q.c * r * n +
                     Q.d * (p * m + q * l) + Q.e * (p * n + r * l) + Q.f * (r * m + q * n) +
                     Q.g * l + Q.h * m + Q.i * n;
    const double C = Q.a * (p * p) + Q.b * (q * q) + Q.c * (r * r) + Q.d * p * q + Q.e * p * r +
                     Q.f * q * r + Q.g * p + Q.h * q + Q.i * r + Q.j;
    const double D = B * B - 4.0 * A * C;
    const double s = sqrt_cr(D);
    const double t = (negative ? (-B - s) : (-B + s)) / (2.0 * A);
    x = t * l + p;
    y = t * m + q;
    z = t * n + r;
    return D > 0.0;
}

// The same intersection for a quadric with b = d = f = h = 0 (no y terms: the reference's
// vertical mirrors before misalignment) or with c = e = f = i = 0 (no z terms). Each skipped term
// is an exact +-0 added to a running sum that is non-zero by then, so the rounded result is the
// one the full expression gives (only the sign of an exactly-zero result could differ).
template <int kFree>  // 1: y-free, 2: z-free
__device__ __forceinline__ bool quadric_hit_sparse(const Quadric& Q, double l, double m, double n, double p,
                                                   double q, double r, bool negative, double& x, double& y,
                                                   double& z) {
    double A, B, C;
    if (kFree == 1) {
        A = Q.a * (l * l) + Q.c * (n * n) + Q.e * n * l;
        B = 2.0 * Q.a * p * l + 2.0 * Q.c * r * n + Q.e * (p * n + r * l) + Q.g * l + Q.i * n;
        C = Q.a * (p * p) + Q.c * (r * r) + Q.e * p * r + Q.g * p + Q.i * r + Q.j;
    } else {
        A = Q.a * (l * l) + Q.b * (m * m) + Q.d * m * l;
        B = 2.0 * Q.a * p * l + 2.0 * Q.b * q * m + Q.d * (p * m + q * l) + Q.g * l + Q.h * m;
        C = Q.a * (p * p) + Q.b * (q * q) + Q.d * p * q + Q.g * p + Q.h * q + Q.j;
    }
    const double D = B * B - 4.0 * A * C;
    const double s = sqrt_cr(D);
    const double t = (negative ? (-B - s) : (-B + s)) / (2.0 * A);
    x = t * l + p;
    y = t * m + q;
    z = t * n + r;
    return D > 0.0;
}

// gradient of the quadric (norm_vector, EllipseRaytrace3D.py:66-68)
__device__ __forceinline__ void quadric_grad(const Quadric& Q, double x, double y, double z, double& nx,
                                             double& ny, double& nz) {
    nx = 2.0 * Q.a * x + Q.d * y + Q.e * z + Q.g;
    ny = 2.0 * Q.b * y + Q.d * x + Q.f * z + Q.h;
    nz = 2.0 * Q.c * z + Q.e * x + Q.f * y + Q.i;
}

// reflect_ray before normalisation (EllipseRaytrace3D.py:51-52)
__device__ __forceinline__ void reflect_raw(double l, double m, double n, double nx, double ny,
                                            double nz, double& rx, double& ry, double& rz) {
    const double A = l * nx + m * ny + n * nz;
    const double A2 = 2.0 * A;
    rx = l - A2 * nx;
    ry = m - A2 * ny;
    rz = n - A2 * nz;
}

struct Mat3 {
    double m[9];
};

// R @ v for a 3x3 R in the order OpenBLAS dgemm forms it for the reference's (3,3) @ (3,N)
// products (AKB_raytrace_20250312.py:929): r0*x, then fma(r1, y, .), then fma(r2, z, .)
__device__ __forceinline__ void matvec(const Mat3& R, double x, double y, double z, double& ox,
                                       double& oy, double& oz) {
    ox = __builtin_fma(R.m[2], z, __builtin_fma(R.m[1], y, R.m[0] * x));
    oy = __builtin_fma(R.m[5], z, __builtin_fma(R.m[4], y, R.m[3] * x));
    oz = __builtin_fma(R.m[8], z, __builtin_fma(R.m[7], y, R.m[6] * x));
}

// plane_ray_intersection (EllipseRaytrace3D.py:150-155)
__device__ __forceinline__ void plane_hit(double g, double h, double i, double j, double l, double m,
                                          double n, double p, double q, double r, double& x,
                                          double& y, double& z) {
    const double t = div_w(-(g * p + h * q + i * r + j), g * l + h * m + i * n);
    x = t * l + p;
    y = t * m + q;
    z = t * n + r;
}

}  // namespace akb

namespace akb {

// ---- numpy-order leaf sums fused into a producer (see akb_leaf_sink in the header) ----
// A producer launched with 256-thread workgroups walks its rays in 256-ray segments (two numpy
// leaves of 128); every thread hands over its ray's NQ quantities and the workgroup writes the
// segment's leaf sums, or the raw values when the segment lies in the short last buffer.
constexpr int kLeafSeg = 256;
constexpr int kNpBuf = 8192;

template <int NQ>
struct LeafLds {
    double v[NQ][kLeafSeg];
};

template <int NQ>
__device__ __forceinline__ void leaf_sink_segment(const akb_leaf_sink& S, LeafLds<NQ>& L, int64_t seg0,
                                                  const double (&v)[NQ], bool valid, int tid) {
    const int64_t full = (S.n / kNpBuf) * kNpBuf;
    if (seg0 >= full) {  // block-uniform: the short last buffer keeps raw values
        if (valid) {
            const int64_t t = seg0 + tid - full;
#pragma unroll
            for (int q = 0; q < NQ; ++q) S.tail[(int64_t)q * kNpBuf + t] = v[q];
        }
        return;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) L.v[q][tid] = v[q];
    __syncthreads();
    if (tid < 16 * NQ) {
        const int q = tid >> 4;
        const int leaf = (tid >> 3) & 1;
        const int j = tid & 7;
        const bool nan0 = (S.nan_mask >> q) & 1;
        const double* p = &L.v[q][leaf * 128 + j];
        // plain sum first: with no NaN among the 16 values it is np.nansum's sum, bit for bit;
        // a NaN result (a NaN input, or inf - inf) re-sums with NaN skipped when the quantity is
        // a nanmean one (for inf - inf that gives the same NaN)
        double r = p[0];
#pragma unroll
        for (int row = 1; row < 16; ++row) r = r + p[row * 8];
        int c = 16;
        // wave-uniform: a per-lane branch is if-converted into 16 compares and 40 selects per
        // segment on every lane
        if (__builtin_expect(__ballot(nan0 && r != r) != 0, 0) && nan0 && r != r) {
            double x = p[0];
            bool bad = x != x;
            r = bad ? 0.0 : x;
            c = bad ? 0 : 1;
            for (int row = 1; row < 16; ++row) {
                x = p[row * 8];
                bad = x != x;
                r = r + (bad ? 0.0 : x);
                c += bad ? 0 : 1;
            }
        }
        // numpy's leaf: ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7))
        r = r + __shfl_xor(r, 1);
        r = r + __shfl_xor(r, 2);
        r = r + __shfl_xor(r, 4);
        c += __shfl_xor(c, 1);
        c += __shfl_xor(c, 2);
        c += __shfl_xor(c, 4);
        if (j == 0) {
            const int64_t nleaves = full / 128;
            const int64_t li = seg0 / 128 + leaf;
            S.leaf_sum[(int64_t)q * nleaves + li] = r;
            S.leaf_cnt[(int64_t)q * nleaves + li] = c;
        }
    }
    __syncthreads();
}
template <int NQ>
__device__ __forceinline__ void leaf_sink_segment(const akb_leaf_sink& S, LeafLds<NQ>& L, int64_t seg0,
                                                  const double (&v)[NQ], bool valid) {
    leaf_sink_segment<NQ>(S, L, seg0, v, valid, (int)threadIdx.x);
}

}  // namespace akb

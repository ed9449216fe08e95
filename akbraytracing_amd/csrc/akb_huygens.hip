// Huygens–Fresnel phase accumulation for gfx950 (the Wavecalc_raytrace_fromData hot loop).
//
//   u[i] = sum_j (u_j dS_j) * exp(-i k r_ij) / r_ij
//   r_ij = sqrt(((x_i - x_j)^2 + (y_i - y_j)^2) + (z_i - z_j)^2)
//
// Reference: compute_u_parallel, Wavecalc_raytrace_fromData_CPU0402.py:71-85 (numba, one target
// per prange iteration, vectorised over sources); the CuPy version materialises a B x M complex
// matrix plus six temporaries per batch (Wavecalc_raytrace_fromData_GPU0402.py:112-120). Here
// nothing is materialised: each lane owns kTPL targets and keeps their sums in registers while the
// workgroup streams source tiles (x, y, z, Re u, Im u) through LDS, so HBM traffic is the source
// set once per workgroup and the kernel is bound by FP64 VALU (sqrt, div, sincos per pair).
//
// r_ij is formed exactly as numpy forms it (no contraction, correctly rounded sqrt), because
// k r ~ 7e10 rad: one ulp of r moves the phase by ~1e-5 rad. The phase -k r is reduced modulo
// pi/2 by a five-piece Cody-Waite split (13-bit pieces: n pi/2 exact for |n| < 2^40, residual
// 2^-65 rad) instead of the library's Payne-Hanek path, and sin / cos come from fdlibm's kernel
// polynomials (< 1 ulp), the quadrant from the rounding shifter's low bits; 1/r comes from the
// distance's own rsq after one Newton step (~1e-13 relative). The complex multiply-accumulate
// uses explicit FMAs. All of it is tolerance-checked against the oracle (numpy's own sum is
// pairwise, so the field is not bitwise anyway).
#include <math.h>

#include "akb_common.h"

namespace akb {

constexpr int kHuyBlock = 256;
constexpr int kHuyTile = 256;  // sources per LDS tile (5 doubles each = 10 KiB)
#ifndef AKB_HUY_TPL
#define AKB_HUY_TPL 2
#endif
constexpr int kTPL = AKB_HUY_TPL;  // targets per lane

// Pair distance and half its reciprocal from one rsq: r = sqrt(x) correctly rounded (sqrt_core's
// sequence, akb_common.h, exact for x in [2^-767, 2^1000] - every distance between points metres
// apart) and h ~ 0.5 / r after one Newton step (relative error ~1e-13, one-signed; the factor 2 is
// applied to the sums once at the end, exactly). x = 0 (a target on a source, where the
// reference's amplitude is inf too) gives r = 0.
__device__ __forceinline__ void dist_half_inv(double x, double& r, double& h) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y;
    h = y * 0.5;
    const double e = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, e, g);
    const double d = __builtin_fma(-g, g, x);
    h = __builtin_fma(h, e, h);
    g = __builtin_fma(d, h, g);
    const double d2 = __builtin_fma(-g, g, x);
    const double out = __builtin_fma(d2, h, g);
    r = x == 0.0 ? 0.0 : out;
}

constexpr double kShift = 0x1.8p52;  // t = x 2/pi + 1.5 2^52 holds rint(x 2/pi) in its low mantissa bits

// phases beyond the fast range (|x 2/pi| >= 2^40; never formed by points metres apart at EUV k):
// the library's sincos (its Payne-Hanek reduction), used only by the fix-up loop after the main one
__device__ __forceinline__ void sincos_slow(double x, double& sn, double& cs) { sincos(x, &sn, &cs); }

// sin and cos of x for |x| < 2^40 pi/2; returns false (values unusable) beyond, where the caller
// takes the library's sincos instead
__device__ __forceinline__ bool sincos_phase_fast(double x, double& sn, double& cs) {
    const double t = __builtin_fma(x, 0x1.45f306dc9c883p-1, kShift);  // rint(x * 2/pi) + shift
    const double q = t - kShift;
    double f = __builtin_fma(-q, 0x1.9220000000000p+0, x);
    f = __builtin_fma(-q, -0x1.2af0000000000p-18, f);
    f = __builtin_fma(-q, 0x1.0b40000000000p-34, f);
    f = __builtin_fma(-q, 0x1.8470000000000p-48, f);
    f = __builtin_fma(-q, -0x1.9d9cceba3f91fp-62, f);
    const double z = f * f;
    // fdlibm __kernel_sin / __kernel_cos on [-pi/4, pi/4]
    const double rs = __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, 0x1.5d93a5acfd57cp-33,
                                    -0x1.ae5e68a2b9cebp-26), 0x1.71de357b1fe7dp-19), -0x1.a01a019c161d5p-13),
                                    0x1.111111110f8a6p-7);
    const double s0 = __builtin_fma(z * f, __builtin_fma(z, rs, -0x1.5555555555549p-3), f);
    const double rc = z * __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z,
                                    -0x1.8fae9be8838d4p-37, 0x1.1ee9ebdb4b1c4p-29), -0x1.27e4f809c52adp-22),
                                    0x1.a01a019cb1590p-16), -0x1.6c16c16c15177p-10), 0x1.555555555554cp-5);
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double c0 = w + (((1.0 - w) - hz) + z * rc);
    // q mod 4 = the shifter's low mantissa bits (2^51 + q, and 2^51 = 0 mod 4, negative q too)
    const unsigned k = (unsigned)__double2loint(t);
    const bool odd = k & 1u;
    const double a = odd ? c0 : s0;  // sin(x) = s0, c0, -s0, -c0 for k = 0..3
    const double b = odd ? s0 : c0;  // cos(x) = c0, -s0, -c0, s0
    // the quadrant's signs as sign-bit flips of the high words (no compares or selects)
    sn = __hiloint2double(__double2hiint(a) ^ (int)((k << 30) & 0x80000000u), __double2loint(a));
    cs = __hiloint2double(__double2hiint(b) ^ (int)(((k + 1u) << 30) & 0x80000000u), __double2loint(b));
    // a NaN phase stays on the fast path (its sums are NaN whatever runs them); only a phase
    // outside the Cody-Waite range sends its target to the fix-up loop
    return !(fabs(q) >= 0x1p40);
}

// one pair's contribution: the distance, 1 / (2 r), the phase -k r and its sincos, the complex
// multiply-accumulate; returns false when the phase left the fast range (the sums then are
// recomputed by the caller's slow loop)
template <bool kSlow>
__device__ __forceinline__ bool pair_add(double px, double py, double pz, double xj, double yj, double zj,
                                         double ur, double ui, double negk, double& ar, double& ai) {
    const double dx = px - xj;
    const double dy = py - yj;
    const double dz = pz - zj;
    double r, amp;  // amp = 1 / (2 r)
    dist_half_inv(dx * dx + dy * dy + dz * dz, r, amp);
    const double ph = negk * r;
    double sn, cs;
    bool ok = true;
    if (kSlow) sincos_slow(ph, sn, cs);
    else ok = sincos_phase_fast(ph, sn, cs);
    const double fr = amp * cs;
    const double fi = amp * sn;
    ar = __builtin_fma(fr, ur, __builtin_fma(-fi, ui, ar));
    ai = __builtin_fma(fr, ui, __builtin_fma(fi, ur, ai));
    return ok;
}

__global__ void __launch_bounds__(kHuyBlock) k_huygens(const double* __restrict__ tx,
                                                       const double* __restrict__ ty,
                                                       const double* __restrict__ tz, int64_t n,
                                                       const double* __restrict__ sx,
                                                       const double* __restrict__ sy,
                                                       const double* __restrict__ sz,
                                                       const double* __restrict__ u, int64_t m,
                                                       int64_t per_split, double negk,
                                                       double* __restrict__ out) {
    __shared__ double s_x[kHuyTile], s_y[kHuyTile], s_z[kHuyTile], s_ur[kHuyTile], s_ui[kHuyTile];
    const int64_t base = (int64_t)blockIdx.x * (kHuyBlock * kTPL);
    double px[kTPL], py[kTPL], pz[kTPL], ar[kTPL], ai[kTPL];
#pragma unroll
    for (int t = 0; t < kTPL; ++t) {
        const int64_t i = base + threadIdx.x + t * kHuyBlock;
        const bool ok = i < n;
        // a lane's slots past the last target sit at the origin: finite pairs, sums never written
        px[t] = ok ? tx[i] : 0.0;
        py[t] = ok ? ty[i] : 0.0;
        pz[t] = ok ? tz[i] : 0.0;
        ar[t] = 0.0;
        ai[t] = 0.0;
    }
    // this workgroup's slice of the sources (blockIdx.y splits M so that small target sets
    // still fill the 256 CUs; the partial sums are added in a fixed order by k_huygens_reduce)
    const int64_t jb = (int64_t)blockIdx.y * per_split;
    const int64_t je = (jb + per_split) < m ? (jb + per_split) : m;
    out += (int64_t)blockIdx.y * 2 * n;
    bool fast[kTPL];  // every pair of target t stayed in the fast phase range
#pragma unroll
    for (int t = 0; t < kTPL; ++t) fast[t] = true;
    for (int64_t j0 = jb; j0 < je; j0 += kHuyTile) {
        const int cnt = (je - j0) < kHuyTile ? (int)(je - j0) : kHuyTile;
        __syncthreads();
        for (int s = threadIdx.x; s < cnt; s += kHuyBlock) {
            const int64_t j = j0 + s;
            s_x[s] = sx[j];
            s_y[s] = sy[j];
            s_z[s] = sz[j];
            s_ur[s] = u[2 * j];
            s_ui[s] = u[2 * j + 1];
        }
        __syncthreads();
        for (int s = 0; s < cnt; ++s) {
            const double xj = s_x[s], yj = s_y[s], zj = s_z[s], ur = s_ur[s], ui = s_ui[s];
#pragma unroll
            for (int t = 0; t < kTPL; ++t)
                fast[t] &= pair_add<false>(px[t], py[t], pz[t], xj, yj, zj, ur, ui, negk, ar[t], ai[t]);
        }
    }
    // a phase beyond the fast reduction's range (|k r| >= 2^40 pi/2: points ~4 km apart at EUV k,
    // never in the reference's geometries): that target's sum again with the library's sincos. Kept
    // out of the loop above so its pair arithmetic carries no branch and no call.
#pragma unroll
    for (int t = 0; t < kTPL; ++t) {
        if (__builtin_expect(!fast[t], 0)) {
            ar[t] = ai[t] = 0.0;
            for (int64_t j = jb; j < je; ++j)
                pair_add<true>(px[t], py[t], pz[t], sx[j], sy[j], sz[j], u[2 * j], u[2 * j + 1], negk, ar[t], ai[t]);
        }
    }
#pragma unroll
    for (int t = 0; t < kTPL; ++t) {
        const int64_t i = base + threadIdx.x + t * kHuyBlock;
        if (i < n) {
            out[2 * i] = 2.0 * ar[t];  // the 1 / (2 r) amplitudes' factor 2, exact
            out[2 * i + 1] = 2.0 * ai[t];
        }
    }
}

// out = sum over splits of the partial fields, in two ordered levels over the 2n interleaved
// doubles (cols): chunks of kRedChunk consecutive splits, then the chunks in order. Each split
// row is read by consecutive lanes. (One lane per target summing all splits kept 4225 lanes busy
// for 3.1 ms on the C2 stage's 9102 splits.) Deterministic: a fixed order for a given split count.
constexpr int kRedChunk = 128;
__global__ void __launch_bounds__(kBlock) k_huygens_reduce(const double* part, int splits, int per,
                                                           int64_t cols, double* out) {
    const int64_t col = blockIdx.x * (int64_t)kBlock + threadIdx.x;
    if (col >= cols) return;
    const int s0 = blockIdx.y * per;
    const int s1 = (s0 + per) < splits ? (s0 + per) : splits;
    double acc = part[(int64_t)s0 * cols + col];
    for (int sp = s0 + 1; sp < s1; ++sp) acc = acc + part[(int64_t)sp * cols + col];
    out[(int64_t)blockIdx.y * cols + col] = acc;
}

__global__ void __launch_bounds__(kBlock) k_scale_field(const double* u, const double* ds, int64_t m,
                                                        double* out) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < m;
         j += (int64_t)gridDim.x * blockDim.x) {
        // complex128 * float64 in numpy: (re*d - im*0, re*0 + im*d)
        const double d = ds[j];
        const double re = u[2 * j], im = u[2 * j + 1];
        out[2 * j] = re * d - im * 0.0;
        out[2 * j + 1] = re * 0.0 + im * d;
    }
}

}  // namespace akb

using namespace akb;

// workgroups of k_huygens the device holds at once (CUs x resident workgroups per CU), 0 if the
// runtime cannot say (no device); a function-local static, initialised once and thread-safely
static int huygens_slots() {
    static const int cached = [] {
        int dev = 0, cus = 0, per_cu = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_huygens, kHuyBlock, 0) == hipSuccess)
            return cus * per_cu;
        (void)hipGetLastError();
        return 0;
    }();
    return cached;
}

#ifndef AKB_HUY_ROUNDS
#define AKB_HUY_ROUNDS 64
#endif
// split partials are capped at this much scratch (2 doubles per target per split): 512 MiB holds
// 7943 splits of the C2 stage's 4225 targets, ~53 rounds
constexpr int64_t kHuyScratchBytes = 512ll << 20;

// how many source splits a launch uses: a whole number of rounds of resident workgroups
// (splits x target blocks = kRounds x the device's slots; measured on the C2 stage: 2052
// workgroups over 1280 slots, 1.6 rounds, 170.7 ms; 1 round 200 ms, 2 rounds 174, 4 142, 8 125,
// 16 118, 64 113.6 ms: finer pieces even out the workgroups' finishing times), at least kMinSplit
// sources per split, and partials within kHuyScratchBytes. The count depends on the device (its
// slots) and on n: a target-sharded caller passes the whole problem's count to every piece
// (akb_huygens_splits) so each target's sum is the same whatever the sharding.
static int huygens_splits(int64_t n, int64_t m) {
    constexpr int64_t kRounds = AKB_HUY_ROUNDS;
    const int64_t per_block = (int64_t)kHuyBlock * kTPL;
    const int64_t tblocks = (n + per_block - 1) / per_block;
    const int slots = huygens_slots();
    const int64_t want = slots > 0 ? (kRounds * slots >= tblocks ? kRounds * slots / tblocks : 1)
                                   : (2048 + tblocks - 1) / tblocks;
    const int64_t kMinSplit = 1024;
    int64_t maxs = (m + kMinSplit - 1) / kMinSplit;
    if (maxs < 1) maxs = 1;
    int64_t s = want < maxs ? want : maxs;
    const int64_t cap = n > 0 ? kHuyScratchBytes / (2 * n * (int64_t)sizeof(double)) : s;
    if (s > cap) s = cap;
    if (s > 65535) s = 65535;
    return (int)(s < 1 ? 1 : s);
}

static int64_t huygens_work_bytes(int64_t n, int splits) {
    if (n <= 0 || splits <= 1) return 0;
    const int64_t chunks = (splits + kRedChunk - 1) / kRedChunk;
    return ((int64_t)splits + (chunks > 1 ? chunks : 0)) * 2 * n * (int64_t)sizeof(double);
}

extern "C" {

int akb_huygens_splits(int64_t n, int64_t m) { return n > 0 && m > 0 ? huygens_splits(n, m) : 1; }

int64_t akb_huygens_work_bytes(int64_t n, int64_t m, int splits) {
    if (n <= 0 || m <= 0) return 0;
    return huygens_work_bytes(n, splits > 0 ? splits : huygens_splits(n, m));
}

int akb_huygens_f64(const double* tx, const double* ty, const double* tz, int64_t n,
                    const double* sx, const double* sy, const double* sz, const double* u_re_im,
                    int64_t m, double k, double* out_re_im, int splits, void* work, void* stream) {
    clear_error();
    AKB_REQUIRE(n >= 0 && m >= 0, "negative size");
    if (n == 0) return AKB_OK;
    AKB_REQUIRE(tx && ty && tz && out_re_im, "null target pointer");
    hipStream_t s = (hipStream_t)stream;
    if (m == 0) {
        AKB_HIP_CHECK(hipMemsetAsync(out_re_im, 0, sizeof(double) * 2 * n, s));
        return AKB_OK;
    }
    AKB_REQUIRE(sx && sy && sz && u_re_im, "null source pointer");
    const int64_t per_block = (int64_t)kHuyBlock * kTPL;
    const int64_t blocks = (n + per_block - 1) / per_block;
    AKB_REQUIRE(blocks < (1LL << 31), "too many targets");
    if (splits <= 0) splits = huygens_splits(n, m);
    AKB_REQUIRE(splits <= 65535, "at most 65535 source splits");
    AKB_REQUIRE(splits == 1 || work != nullptr, "work buffer required (akb_huygens_work_bytes)");
    const int64_t per_split = (m + splits - 1) / splits;
    double* dst = splits == 1 ? out_re_im : (double*)work;
    // numpy's phase is (-k) * dist; negate the scalar once (exact)
    k_huygens<<<dim3((unsigned)blocks, splits), kHuyBlock, 0, s>>>(tx, ty, tz, n, sx, sy, sz, u_re_im,
                                                                   m, per_split, -k, dst);
    int st = launch_status("k_huygens");
    if (st || splits == 1) return st;
    const int64_t cols = 2 * n;
    const unsigned bx = (unsigned)((cols + kBlock - 1) / kBlock);
    const int chunks = (splits + kRedChunk - 1) / kRedChunk;
    double* lvl = chunks > 1 ? dst + (int64_t)splits * cols : out_re_im;  // chunk sums after the partials
    k_huygens_reduce<<<dim3(bx, (unsigned)chunks), kBlock, 0, s>>>(dst, splits, kRedChunk, cols, lvl);
    if ((st = launch_status("k_huygens_reduce")) || chunks == 1) return st;
    k_huygens_reduce<<<dim3(bx, 1), kBlock, 0, s>>>(lvl, chunks, chunks, cols, out_re_im);
    return launch_status("k_huygens_reduce");
}

int akb_scale_field_f64(const double* u_re_im, const double* ds, int64_t m, double* out_re_im,
                        void* stream) {
    clear_error();
    AKB_REQUIRE(m >= 0, "negative size");
    if (m == 0) return AKB_OK;
    AKB_REQUIRE(u_re_im && ds && out_re_im, "null pointer");
    k_scale_field<<<grid_for(m), kBlock, 0, (hipStream_t)stream>>>(u_re_im, ds, m, out_re_im);
    return launch_status("k_scale_field");
}

}  // extern "C"

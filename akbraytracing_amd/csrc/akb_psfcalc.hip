// psf_calc's pupil preparation for gfx950 (AKB_raytrace_20250312.py:1121-1188): the rotation
// estimate's per-column first valid row, and rotate_with_nan(order=3) — scipy.ndimage.rotate
// (reshape=False, mode 'constant') of the NaN-filled map and of its finite mask, divided, NaN
// where the rotated mask < 0.5.
//
// scipy's order-3 rotate is a cubic B-spline prefilter along each axis followed by a 4 x 4
// B-spline sum at each output pixel's source point (oracle/psfcalc.py states the algorithm and
// its boundary rules). The maps are small (65^2 .. 1k^2): one thread per line for the recursive
// prefilter, one thread per output pixel for the interpolation, both arrays at once.
#include <type_traits>

#include "akb_common.h"
#include "akb_pairwise.h"

namespace akb {

__global__ void k_first_valid_rows(const double* __restrict__ m, int ny, int nx, int32_t* __restrict__ out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nx) return;
    int r = 0;
    while (r < ny && m[(int64_t)r * nx + c] != m[(int64_t)r * nx + c]) ++r;
    out[c] = r < ny ? r : -1;
}

// coef[0] = NaN-filled map, coef[1] = its finite mask (as floats)
__global__ void k_nan_split(const double* __restrict__ m, int64_t n, double* __restrict__ coef) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double v = m[i];
        const bool nan = v != v;
        coef[i] = nan ? 0.0 : v;
        coef[n + i] = nan ? 0.0 : 1.0;
    }
}

// scipy spline_filter1d(order 3) along each line of one axis: gain 6, mirror-symmetric causal
// initialisation, causal pass, anti-causal initialisation and pass (the order of oracle/psfcalc.py)
__device__ void spline_line(double* c, int n, int64_t s) {
    const double z = sqrt(3.0) - 2.0;
    const double gain = (1.0 - z) * (1.0 - 1.0 / z);
    for (int i = 0; i < n; ++i) c[i * s] = c[i * s] * gain;
    if (n == 1) return;
    const double zn1 = pow(z, (double)(n - 1));
    double c0 = c[0] + zn1 * c[(n - 1) * s];
    double zi = z;
    for (int i = 1; i < n - 1; ++i) {
        c0 += zi * (c[i * s] + zn1 * c[(n - 1 - i) * s]);
        zi *= z;
    }
    c[0] = c0 / (1.0 - zn1 * zn1);
    for (int i = 1; i < n; ++i) c[i * s] += z * c[(i - 1) * s];
    c[(n - 1) * s] = (z * c[(n - 2) * s] + c[(n - 1) * s]) * z / (z * z - 1.0);
    for (int i = n - 2; i >= 0; --i) c[i * s] = z * (c[(i + 1) * s] - c[i * s]);
}

__global__ void k_spline_lines(double* __restrict__ coef, int ny, int nx, int axis) {
    // blockIdx.y: which array (map, mask); one thread per line
    const int line = blockIdx.x * blockDim.x + threadIdx.x;
    const int nlines = axis == 0 ? nx : ny;
    if (line >= nlines) return;
    double* base = coef + (int64_t)blockIdx.y * ny * nx;
    spline_line(base + (axis == 0 ? line : (int64_t)line * nx), axis == 0 ? ny : nx, axis == 0 ? nx : 1);
}

__device__ __forceinline__ int mirror_index(int i, int n) {
    if (n == 1) return 0;
    const int p = 2 * n - 2;
    i = abs(i) % p;
    return i >= n ? p - i : i;
}

__device__ __forceinline__ void bspline3(double t, double (&w)[4]) {
    const double u = 1.0 - t;
    w[0] = u * u * u / 6.0;
    w[1] = (4.0 - 6.0 * t * t + 3.0 * (t * t * t)) / 6.0;
    w[2] = (1.0 + 3.0 * t + 3.0 * t * t - 3.0 * (t * t * t)) / 6.0;
    w[3] = t * t * t / 6.0;
}

struct RotArgs {
    const double* coef;  // (2, ny, nx): prefiltered map, prefiltered mask
    int ny, nx;
    double m00, m01, m10, m11, off0, off1;
    double* rotated;  // nm, NaN outside the rotated mask
    double* opd_m;    // rotated * 1e-9 (or NULL)
};

__device__ __forceinline__ void rotate_pixel(const RotArgs& a, int64_t k) {
    const int64_t total = (int64_t)a.ny * a.nx;
    {
        const int i = (int)(k / a.nx), j = (int)(k - (int64_t)i * a.nx);
        const double y = a.m00 * i + a.m01 * j + a.off0;
        const double x = a.m10 * i + a.m11 * j + a.off1;
        double f = 0.0, msk = 0.0;
        if (y >= 0.0 && y <= a.ny - 1 && x >= 0.0 && x <= a.nx - 1) {
            const double fy = floor(y), fx = floor(x);
            double wy[4], wx[4];
            bspline3(y - fy, wy);
            bspline3(x - fx, wx);
            const int iy0 = (int)fy - 1, ix0 = (int)fx - 1;
            const double* cm = a.coef + total;
            for (int p = 0; p < 4; ++p) {
                const int64_t row = (int64_t)mirror_index(iy0 + p, a.ny) * a.nx;
                for (int q = 0; q < 4; ++q) {
                    const int64_t idx = row + mirror_index(ix0 + q, a.nx);
                    const double w = wy[p] * wx[q];
                    f = f + w * a.coef[idx];
                    msk = msk + w * cm[idx];
                }
            }
        }
        double r = f / fmax(msk, 1e-12);
        if (msk < 0.5) r = __builtin_nan("");
        a.rotated[k] = r;
        if (a.opd_m) a.opd_m[k] = r * 1e-9;
    }
}

__global__ void k_rotate_cubic(RotArgs a) {
    const int64_t total = (int64_t)a.ny * a.nx;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < total; k += (int64_t)gridDim.x * blockDim.x)
        rotate_pixel(a, k);
}

// rotate_with_nan's interpolation after k_pupil_post: scipy.ndimage.rotate's matrix and offsets
// from its parameter block (cos, sin, offsets at [13 .. 17), akb_raytrace.h)
__global__ void k_rotate_post(const double* coef, int ny, int nx, const double* P, double* rotated, double* opd) {
    AKB_CHAIN_PRIORITY();
    const RotArgs ra{coef, ny, nx, P[13], P[14], -P[14], P[13], P[15], P[16], rotated, opd};
    const int64_t total = (int64_t)ny * nx;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < total; k += (int64_t)gridDim.x * blockDim.x)
        rotate_pixel(ra, k);
}

// ---- plane_correction_with_nan_and_outlier_filter (ref :9630-9693) and match_legendre (:59-73) ----
//
// Both are least-squares / projection steps over a 2-D map with NaNs. The device forms the sums
// (per-workgroup partials in a fixed order, then one workgroup adds them in order: deterministic),
// the host solves the 5 x 5 / 3 x 3 normal equations. Basis: 1, X, Y, X^2, Y^2 with X, Y the
// column / row index centred and scaled to [-1, 1] (the same least-squares plane as the
// reference's x, y indices, better conditioned).

constexpr int kMomMax = 21;  // 15 (upper triangle of 5 x 5) + 5 (rhs) + 1 (count)

struct MomArgs {
    const double* z;
    int ny, nx;
    int nb;                 // basis size: 5 (quadratic) or 3 (plane)
    const double* coef;     // NULL: all finite points; else keep |z - model(coef, 5 terms)| < thr
    double thr;
    int mode;               // 0: normal-equation sums; 1: residual sum; 2: residual sum of squares
    double mean;            // mode 2: residual mean
    double* part;           // (gridDim.x, kMomMax)
};

// basis5 from per-axis tables (the same X, Y values; tables only for axes of up to kPostBasisMax)
constexpr int kPostBasisMax = 256;
__device__ __forceinline__ void basis5_tab(const double* bX, const double* bY, int i, int j, int ny, int nx,
                                           double (&f)[5]) {
    const double X = nx <= kPostBasisMax && ny <= kPostBasisMax ? bX[j] : (nx > 1 ? (2.0 * j - (nx - 1)) / (double)(nx - 1) : 0.0);
    const double Y = nx <= kPostBasisMax && ny <= kPostBasisMax ? bY[i] : (ny > 1 ? (2.0 * i - (ny - 1)) / (double)(ny - 1) : 0.0);
    f[0] = 1.0;
    f[1] = X;
    f[2] = Y;
    f[3] = X * X;
    f[4] = Y * Y;
}

__device__ __forceinline__ void basis5(int i, int j, int ny, int nx, double (&f)[5]) {
    const double X = nx > 1 ? (2.0 * j - (nx - 1)) / (double)(nx - 1) : 0.0;
    const double Y = ny > 1 ? (2.0 * i - (ny - 1)) / (double)(ny - 1) : 0.0;
    f[0] = 1.0;
    f[1] = X;
    f[2] = Y;
    f[3] = X * X;
    f[4] = Y * Y;
}

__global__ void __launch_bounds__(kBlock) k_moments(MomArgs a) {
    __shared__ double red[kBlock / 64][kMomMax];
    double acc[kMomMax];
#pragma unroll
    for (int q = 0; q < kMomMax; ++q) acc[q] = 0.0;
    const int64_t total = (int64_t)a.ny * a.nx;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < total; k += (int64_t)gridDim.x * blockDim.x) {
        const double z = a.z[k];
        if (z != z) continue;
        const int i = (int)(k / a.nx), j = (int)(k - (int64_t)i * a.nx);
        double f[5];
        basis5(i, j, a.ny, a.nx, f);
        double res = 0.0;
        if (a.coef || a.mode > 0) {
            double m = 0.0;
            for (int t = 0; t < 5; ++t) m = __builtin_fma(a.coef[t], f[t], m);
            res = z - m;
            if (a.mode == 0 && !(fabs(res) < a.thr)) continue;
        }
        if (a.mode == 1) {
            acc[0] += res;
            acc[20] += 1.0;
        } else if (a.mode == 2) {
            const double d = res - a.mean;
            acc[0] = __builtin_fma(d, d, acc[0]);
            acc[20] += 1.0;
        } else {
            const bool quad = a.nb == 5;
#pragma unroll
            for (int r = 0; r < 5; ++r) {
#pragma unroll
                for (int c = r; c < 5; ++c) {
                    const int q = r * 5 - r * (r - 1) / 2 + (c - r);  // upper-triangle slot
                    if (quad || c < 3) acc[q] = __builtin_fma(f[r], f[c], acc[q]);
                }
                if (quad || r < 3) acc[15 + r] = __builtin_fma(f[r], z, acc[15 + r]);
            }
            acc[20] += 1.0;
        }
    }
#pragma unroll
    for (int q = 0; q < kMomMax; ++q)
        for (int off = 32; off > 0; off >>= 1) acc[q] += __shfl_down(acc[q], off);
    if ((threadIdx.x & 63) == 0)
        for (int q = 0; q < kMomMax; ++q) red[threadIdx.x >> 6][q] = acc[q];
    __syncthreads();
    if (threadIdx.x < kMomMax) {
        double v = red[0][threadIdx.x];
        for (int w = 1; w < kBlock / 64; ++w) v += red[w][threadIdx.x];
        a.part[(int64_t)blockIdx.x * kMomMax + threadIdx.x] = v;
    }
}

__global__ void k_moments_final(const double* part, int nparts, double* out) {
    const int q = threadIdx.x;
    if (q >= kMomMax) return;
    double v = 0.0;
    for (int b = 0; b < nparts; ++b) v += part[(int64_t)b * kMomMax + q];
    out[q] = v;
}

// out = z - plane(coef, 3 terms); NaN where z is NaN
__global__ void __launch_bounds__(kBlock) k_plane_subtract(const double* __restrict__ z, int ny, int nx,
                                                           const double* __restrict__ coef, double* __restrict__ out) {
    const int64_t total = (int64_t)ny * nx;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < total; k += (int64_t)gridDim.x * blockDim.x) {
        const int i = (int)(k / nx), j = (int)(k - (int64_t)i * nx);
        double f[5];
        basis5(i, j, ny, nx, f);
        const double m = __builtin_fma(coef[2], f[2], __builtin_fma(coef[1], f[1], coef[0] * f[0]));
        const double v = z[k];
        out[k] = v != v ? v : v - m;
    }
}

// ---- the pupil's whole post-processing in one workgroup (no host round trip) ----
//
// The driver's chain from the gridded Wave2 map to compute_psf_fft's input
// (AKB_raytrace_20250312.py:3690-3700, :9630-9693, :1121-1188): matrixWave2 -= np.nanmean,
// plane_correction_with_nan_and_outlier_filter (the moments and normal-equation solves of
// pupilmap._plane_corrections, on the device), psf_calc's rotation estimate, and rotate_with_nan
// (order 3) with scipy.ndimage.rotate's matrix from cephes' cosdg / sindg. One 1024-thread
// workgroup does it all for maps of up to 65536 points (the pipelined 128^2 pupil): each step is a
// workgroup pass over the map in L2 with a fixed-order reduction, so a pipelined caller queues the
// PSF behind it with no host synchronisation. The nanmean is numpy's (pairwise over 8192-element
// buffers, left to right); the moments' association differs from k_moments (rounding-level
// differences, tests hold the maps to 1e-12 of the range).

// cephes sindg / cosdg (degrees; the functions scipy.ndimage.rotate calls for its matrix, scipy
// 1.15 special/xsf/cephes/sindg.h): octant reduction in degrees, then the cephes minimax polynomials
// on [0, pi/4]; every product and sum rounded on its own, as the host library evaluates them.
__device__ __constant__ double kSinCof[6] = {1.58962301572218447952E-10, -2.50507477628503540135E-8,
                                             2.75573136213856773549E-6,  -1.98412698295895384658E-4,
                                             8.33333333332211858862E-3,  -1.66666666666666307295E-1};
__device__ __constant__ double kCosCof[7] = {1.13678171382044553091E-11, -2.08758833757683644217E-9,
                                             2.75573155429816611547E-7,  -2.48015872936186303776E-5,
                                             1.38888888888806666760E-3,  -4.16666666666666348141E-2,
                                             4.99999999999999999798E-1};

__device__ __forceinline__ double horner(double x, const double* c, int deg) {
    double r = c[0];
    for (int i = 1; i <= deg; ++i) r = r * x + c[i];
    return r;
}

// octant of |x| degrees (cephes' reduction): returns j in 0..3 and sets y to the multiple of 45
// taken off, flipping *neg for the octants 4..7
__device__ __forceinline__ int deg_octant(double x, double& y, bool& flip) {
    y = floor(x / 45.0);
    double z = ldexp(y, -4);
    z = floor(z);
    z = y - ldexp(z, 4);
    int j = (int)z;
    if (j & 1) {
        j += 1;
        y += 1.0;
    }
    j &= 7;
    flip = j > 3;
    return flip ? j - 4 : j;
}

__device__ double sin_deg(double x) {
    bool neg = x < 0;
    if (neg) x = -x;
    if (x > 1.0e14) return 0.0;
    double y;
    bool flip;
    const int j = deg_octant(x, y, flip);
    if (flip) neg = !neg;
    double z = x - y * 45.0;
    z = z * 1.74532925199432957692E-2;
    const double zz = z * z;
    double r = (j == 1 || j == 2) ? 1.0 - zz * horner(zz, kCosCof, 6) : z + z * (zz * horner(zz, kSinCof, 5));
    return neg ? -r : r;
}

__device__ double cos_deg(double x) {
    if (x < 0) x = -x;
    if (x > 1.0e14) return 0.0;
    double y;
    bool flip;
    const int j = deg_octant(x, y, flip);
    bool neg = flip;
    if (j > 1) neg = !neg;
    double z = x - y * 45.0;
    z = z * 1.74532925199432957692E-2;
    const double zz = z * z;
    double r = (j == 1 || j == 2) ? z + z * (zz * horner(zz, kSinCof, 5)) : 1.0 - zz * horner(zz, kCosCof, 6);
    return neg ? -r : r;
}

// A x = b by Gaussian elimination with partial pivoting (the largest magnitude in the column,
// the first on ties, as LAPACK's dgetf2 picks); A row-major n x n, solution in b. false: singular.
__device__ bool solve_small(double* A, double* b, int n) {
    for (int k = 0; k < n; ++k) {
        int p = k;
        for (int i = k + 1; i < n; ++i)
            if (fabs(A[i * n + k]) > fabs(A[p * n + k])) p = i;
        if (A[p * n + k] == 0.0) return false;
        if (p != k) {
            for (int j = 0; j < n; ++j) {
                const double t = A[k * n + j];
                A[k * n + j] = A[p * n + j];
                A[p * n + j] = t;
            }
            const double t = b[k];
            b[k] = b[p];
            b[p] = t;
        }
        for (int i = k + 1; i < n; ++i) {
            const double l = A[i * n + k] / A[k * n + k];
            for (int j = k; j < n; ++j) A[i * n + j] = A[i * n + j] - l * A[k * n + j];
            b[i] = b[i] - l * b[k];
        }
    }
    for (int k = n - 1; k >= 0; --k) {
        double v = b[k];
        for (int j = k + 1; j < n; ++j) v = v - A[k * n + j] * b[j];
        b[k] = v / A[k * n + k];
    }
    return true;
}

// solve_small in registers for a fixed n (every index a compile-time one: the pivot row swap is a
// select per row), the same operations in the same order - thread-local arrays with runtime indices
// would live in scratch memory, a global-memory round trip per access on this one-thread path
template <int N>
__device__ __forceinline__ bool solve_small_reg(double (&A)[N][N], double (&b)[N]) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        int p = k;
        double best = fabs(A[k][k]);
#pragma unroll
        for (int i = k + 1; i < N; ++i)
            if (fabs(A[i][k]) > best) {
                p = i;
                best = fabs(A[i][k]);
            }
        // the pivot row (the largest magnitude in column k, the first on ties) into row k: a
        // conditional exchange of rows k and i for each i, on a flag the compiler cannot relate to
        // p (else it folds the selects into a row index - an array in scratch memory, a memory
        // round trip per pivot on this one-thread path)
#pragma unroll
        for (int i = k + 1; i < N; ++i) {
            int sw = i == p;
            asm volatile("" : "+v"(sw));
#pragma unroll
            for (int j = 0; j < N; ++j) {
                const double rk = A[k][j], ri = A[i][j];
                A[k][j] = sw ? ri : rk;
                A[i][j] = sw ? rk : ri;
            }
            const double bk = b[k], bi = b[i];
            b[k] = sw ? bi : bk;
            b[i] = sw ? bk : bi;
        }
        if (A[k][k] == 0.0) ok = false;
#pragma unroll
        for (int i = k + 1; i < N; ++i) {
            const double l = A[i][k] / A[k][k];
#pragma unroll
            for (int j = k; j < N; ++j) A[i][j] = A[i][j] - l * A[k][j];
            b[i] = b[i] - l * b[k];
        }
    }
#pragma unroll
    for (int k = N - 1; k >= 0; --k) {
        double v = b[k];
#pragma unroll
        for (int j = k + 1; j < N; ++j) v = v - A[k][j] * b[j];
        b[k] = v / A[k][k];
    }
    return ok;
}

// ---- the post: one workgroup over the map (in LDS when it fits) - nanmean, the plane fits, the NaN
// split, the rotation estimate - then the B-spline prefilter (k_spline_post: a workgroup per array,
// both axes in LDS, four threads per line) and the rotation (k_rotate_post). A grid of workgroups
// with a grid barrier between the phases was measured at ~10 us per barrier (the device-scope
// release and acquire around each), three times the one workgroup's phases.
constexpr int kPostThreads = 1024;
constexpr int64_t kPostMax = 65536;  // map points the post handles
constexpr int kPostFuse = 128;       // arrays up to 128 x 128: the prefilter in LDS, both axes in one launch

struct PostArgs {
    const double* m;     // (ny, nx) gridded map (NaN outside the hull)
    int ny, nx;
    double sigma;        // the outlier filter's threshold in standard deviations (3)
    double* corrected;   // matrixWave2_Corrected
    double* coef;        // work: (2, ny, nx) prefilter coefficients (the NaN split)
    double* params;      // out, kPostParams doubles (layout in akb_raytrace.h)
    unsigned long long* clocks;  // work: the wall clock (100 MHz) at the phase ends (diagnostics)
};

// one DPP step of a wave reduction on a double: v + (v moved by the DPP control), rows outside
// row_mask adding zero
template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ double dpp_add(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), kCtrl, kRowMask, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), kCtrl, kRowMask, 0xf, false);
    return v + __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// the wave's sum in lane 63 (pairs, quads, rows of 16 by rotation, then the rows by broadcast: DPP
// moves, no LDS traffic; a fixed order, so the same bits every time)
__device__ __forceinline__ double wave_sum_dpp(double v) {
    v = dpp_add<0xb1>(v);        // quad_perm [1, 0, 3, 2]
    v = dpp_add<0x4e>(v);        // quad_perm [2, 3, 0, 1]
    v = dpp_add<0x124>(v);       // row_ror:4
    v = dpp_add<0x128>(v);       // row_ror:8
    v = dpp_add<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
    v = dpp_add<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3
    return v;
}

// fixed-order workgroup sum of q values per thread (DPP within the waves, then the waves in order)
template <int Q>
__device__ __forceinline__ void block_sum(double (&acc)[Q], double (*red)[Q]) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < Q; ++q) acc[q] = wave_sum_dpp(acc[q]);
    if (lane == 63)
#pragma unroll
        for (int q = 0; q < Q; ++q) red[w][q] = acc[q];
    __syncthreads();
    if (threadIdx.x < Q) {
        double v = red[0][threadIdx.x];
        for (int k = 1; k < kPostThreads / 64; ++k) v += red[k][threadIdx.x];
        red[0][threadIdx.x] = v;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < Q; ++q) acc[q] = red[0][q];
    __syncthreads();
}

// LDS of the post: the map for the nanmean and the moment passes (maps of up to 16384 points; larger
// ones are read from global memory and `corrected`)
constexpr int kPostLds = 16384;

// a thread's map points k = tid + q kPostThreads as (row, column), stepped without divisions
struct PostIdx {
    int i, j, di, dj, nx;
    __device__ PostIdx(int tid, int nx_) : nx(nx_) {
        i = tid / nx_;
        j = tid - i * nx_;
        di = kPostThreads / nx_;
        dj = kPostThreads - di * nx_;
    }
    __device__ void next() {
        i += di;
        j += dj;
        if (j >= nx) {
            j -= nx;
            ++i;
        }
    }
};

// spline_line's arithmetic on a line in LDS (stride s), in chunks of kCh points: each chunk's values
// are read at once (independent LDS reads), the pass runs on them in registers with the running
// value carried across chunks, and the chunk is written back - the same operations in the same
// order as spline_line, so the same bits, without an LDS write-then-read round trip per point
template <int kCh>
__device__ void spline_line_lds(double* c, int n, int s) {
    const double z = sqrt(3.0) - 2.0;
    const double gain = (1.0 - z) * (1.0 - 1.0 / z);
    double v[kCh], u[kCh];
    for (int i0 = 0; i0 < n; i0 += kCh) {  // the gain
        const int m = min(kCh, n - i0);
#pragma unroll
        for (int k = 0; k < kCh; ++k)
            if (k < m) v[k] = c[(i0 + k) * s];
#pragma unroll
        for (int k = 0; k < kCh; ++k)
            if (k < m) c[(i0 + k) * s] = v[k] * gain;
    }
    if (n == 1) return;
    const double zn1 = pow(z, (double)(n - 1));
    // the mirror-symmetric causal initialisation: c0 = c[0] + zn1 c[n-1] + sum_i z^i (c[i] + zn1 c[n-1-i])
    double c0 = c[0] + zn1 * c[(n - 1) * s];
    double zi = z;
    for (int i0 = 1; i0 < n - 1; i0 += kCh) {
        const int m = min(kCh, n - 1 - i0);
#pragma unroll
        for (int k = 0; k < kCh; ++k)
            if (k < m) {
                v[k] = c[(i0 + k) * s];
                u[k] = c[(n - 1 - i0 - k) * s];
            }
#pragma unroll
        for (int k = 0; k < kCh; ++k)
            if (k < m) {
                c0 += zi * (v[k] + zn1 * u[k]);
                zi *= z;
            }
    }
    double prev = c0 / (1.0 - zn1 * zn1);
    c[0] = prev;
    for (int i0 = 1; i0 < n; i0 += kCh) {  // causal: c[i] += z c[i-1]
        const int m = min(kCh, n - i0);
#pragma unroll
        for (int k = 0; k < kCh; ++k)
            if (k < m) v[k] = c[(i0 + k) * s];
#pragma unroll
        for (int k = 0; k < kCh; ++k)
            if (k < m) {
                v[k] += z * prev;
                prev = v[k];
            }
#pragma unroll
        for (int k = 0; k < kCh; ++k)
            if (k < m) c[(i0 + k) * s] = v[k];
    }
    // anti-causal: c[n-1] from the last two, then c[i] = z (c[i+1] - c[i]) downwards
    double next = (z * c[(n - 2) * s] + prev) * z / (z * z - 1.0);
    c[(n - 1) * s] = next;
    for (int i0 = n - 2; i0 >= 0; i0 -= kCh) {
        const int m = min(kCh, i0 + 1);
#pragma unroll
        for (int k = 0; k < kCh; ++k)
            if (k < m) v[k] = c[(i0 - k) * s];
#pragma unroll
        for (int k = 0; k < kCh; ++k)
            if (k < m) {
                v[k] = z * (next - v[k]);
                next = v[k];
            }
#pragma unroll
        for (int k = 0; k < kCh; ++k)
            if (k < m) c[(i0 - k) * s] = v[k];
    }
}

// spline_filter1d along one axis in LDS: a workgroup of 256 threads takes kSplineLines lines of
// one array (blockIdx.y: map, mask), loads them with all its threads (eight independent loads in
// flight per thread), runs each line's recursion on one thread (spline_line_lds), stores them back.
// Lines of up to 256 points.
constexpr int kSplineLines = 16, kSplineMaxLen = 256, kSplineThreads = 256;
__global__ void __launch_bounds__(kSplineThreads) k_spline_block(double* __restrict__ coef, int ny, int nx, int axis) {
    __shared__ double buf[kSplineMaxLen * (kSplineLines + 1)];
    const int nlines = axis == 0 ? nx : ny, len = axis == 0 ? ny : nx;
    const int l0 = blockIdx.x * kSplineLines, nl = min(kSplineLines, nlines - l0);
    double* base = coef + (int64_t)blockIdx.y * ny * nx;
    const int P = kSplineLines + 1;  // buf[i * P + l]: point i of line l
    const int total = len * nl;
    auto gidx = [&](int e, int& bi) {
        int i, l;
        if (axis == 0) { i = e / nl; l = e - (e / nl) * nl; }  // columns: read along rows (coalesced pieces)
        else { l = e / len; i = e - (e / len) * len; }         // rows: read along the row
        bi = i * P + l;
        return axis == 0 ? (int64_t)i * nx + (l0 + l) : (int64_t)(l0 + l) * nx + i;
    };
    for (int e0 = 0; e0 < total; e0 += 8 * kSplineThreads) {
        double t[8];
        int bi[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int e = e0 + k * kSplineThreads + (int)threadIdx.x;
            if (e < total) t[k] = base[gidx(e, bi[k])];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (e0 + k * kSplineThreads + (int)threadIdx.x < total) buf[bi[k]] = t[k];
    }
    __syncthreads();
    if ((int)threadIdx.x < nl) spline_line_lds<16>(buf + threadIdx.x, len, P);
    __syncthreads();
    for (int e = threadIdx.x; e < total; e += kSplineThreads) {
        int bi;
        const int64_t gi = gidx(e, bi);
        base[gi] = buf[bi];
    }
}

// spline_filter1d's recursions on a line in LDS (stride s) split over P consecutive lanes of a wave
// (sub: the lane's segment of ceil(n / P) <= SEG points, held in registers: one batch of LDS reads,
// one of writes): the gain; the mirror-symmetric initial sum as per-segment parts added in segment
// order; the causal pass c[i] += z c[i-1] run per segment from zero and corrected by z^(i - b0 + 1)
// times the true value before the segment (the carries passed up the segments); the anti-causal
// pass c[i] = z (c[i+1] - c[i]) likewise downwards. The same recursions as spline_line, a different
// rounding order (~1e-16 relative; |z| = 0.27), a P-th of the sequential steps.
__device__ __forceinline__ double zpow(double z, int k) {  // z^k by binary powering (k >= 0)
    double r = 1.0, b = z;
    while (k > 0) {
        if (k & 1) r *= b;
        b *= b;
        k >>= 1;
    }
    return r;
}

// a lane group's neighbour values by DPP row shifts (P lanes, P dividing 16): the value of lane
// sub - 1 (0 for sub 0) and of lane sub + 1 (0 for the top lane)
template <int kCtrl>
__device__ __forceinline__ double dpp_mov(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), kCtrl, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), kCtrl, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
template <int P>
__device__ __forceinline__ double seg_from_below(double v, int sub) {
    const double t = dpp_mov<0x111>(v);  // row_shr:1
    return sub == 0 ? 0.0 : t;
}
template <int P>
__device__ __forceinline__ double seg_from_above(double v, int sub) {
    const double t = dpp_mov<0x101>(v);  // row_shl:1
    return sub == P - 1 ? 0.0 : t;
}

template <int P, int SEG, int s>  // s: the line's stride in LDS (a constant: every read an immediate offset)
__device__ void spline_line_reg(double* c, int n, int sub, unsigned long long* ck = nullptr) {
    const double z = sqrt(3.0) - 2.0;
    const double gain = (1.0 - z) * (1.0 - 1.0 / z);
    const int lane = threadIdx.x & 63, base = lane & ~(P - 1);
    const int seg = (n + P - 1) / P;
    const int b0 = min(n, sub * seg), len = min(n, b0 + seg) - b0;
    double v[SEG];
#pragma unroll
    for (int k = 0; k < SEG; ++k) v[k] = k < len ? c[(b0 + k) * s] * gain : 0.0;
    // the gained values at 0, n - 2 and n - 1 (their owners' registers, summed over the group: the
    // others add zeros)
    auto at = [&](int idx) {  // one read from the owner's registers
        double own = 0.0;
#pragma unroll
        for (int k = 0; k < SEG; ++k)
            if (k < len && b0 + k == idx) own = v[k];
        return __shfl(own, base + idx / seg);
    };
    if (ck) ck[0] = wall_clock64();
    if (n > 1) {
        const double zn1 = zpow(z, n - 1);
        // the mirror-symmetric initial sum: c0 = c[0] + zn1 c[n-1] + sum_{i=1}^{n-2} z^i (c[i] + zn1 c[n-1-i])
        double part = 0.0;
        {
            double zi = zpow(z, b0);
#pragma unroll
            for (int k0 = 0; k0 < SEG; k0 += 8) {  // the mirror values eight reads at a time
                double mir[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int i = b0 + k0 + k;
                    mir[k] = (k0 + k < len && i >= 1 && i <= n - 2) ? c[(n - 1 - i) * s] * gain : 0.0;
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int i = b0 + k0 + k;
                    if (k0 + k < len && i >= 1 && i <= n - 2) part += zi * (v[k0 + k] + zn1 * mir[k]);
                    zi *= z;
                }
            }
        }
        // the parts summed in segment order (((0 + p0) + p1) + ...): passed up the group, then read
        // from its top lane
        double run = 0.0;
#pragma unroll
        for (int q = 0; q < P - 1; ++q) run = seg_from_below<P>(run + part, sub);
        const double tot = __shfl(run + part, base + P - 1);
        const double y0 = (at(0) + zn1 * at(n - 1) + tot) / (1.0 - zn1 * zn1);
        const double zl = zpow(z, len);  // z^(segment length), 1 for an empty segment
        if (ck) ck[1] = wall_clock64();
        // causal
        double u = 0.0;
#pragma unroll
        for (int k = 0; k < SEG; ++k)
            if (k < len) {
                u = k == 0 ? (b0 == 0 ? y0 : v[0]) : v[k] + z * u;
                v[k] = u;
            }
        // the true value at b0 - 1: e_0 = 0, e_{q+1} = u_q + z^len_q e_q, passed up the group one lane a
        // step (after step s lanes 0 .. s + 1 hold theirs)
        double ein = 0.0;
#pragma unroll
        for (int q = 0; q < P - 1; ++q) ein = seg_from_below<P>(u + zl * ein, sub);
        {
            double zk = z;
#pragma unroll
            for (int k = 0; k < SEG; ++k)
                if (k < len) {
                    v[k] = v[k] + zk * ein;
                    zk *= z;
                }
        }
        if (ck) ck[2] = wall_clock64();
        // anti-causal
        const double next = (z * at(n - 2) + at(n - 1)) * z / (z * z - 1.0);
        double w = 0.0;
        const bool top = b0 + len == n;
#pragma unroll
        for (int k = SEG - 1; k >= 0; --k)
            if (k < len) {
                w = (top && k == len - 1) ? next : z * (w - v[k]);
                v[k] = w;
            }
        // the true value at b0 + len, passed down the group likewise
        double bin = 0.0;
#pragma unroll
        for (int q = 0; q < P - 1; ++q) bin = seg_from_above<P>(w + zl * bin, sub);
        {
            double zk = z;
#pragma unroll
            for (int k = SEG - 1; k >= 0; --k)
                if (k < len) {
                    v[k] = v[k] + zk * bin;
                    zk *= z;
                }
        }
    }
    wave_sync();  // every lane's reads (the mirror values) are done before any write
#pragma unroll
    for (int k = 0; k < SEG; ++k)
        if (k < len) c[(b0 + k) * s] = v[k];
}

// the post's B-spline prefilter for arrays of up to kPostFuse x kPostFuse: workgroup 0 the map,
// 1 the mask, each array in LDS (row pitch kPostFuse + 1), both axes, eight lanes per line
constexpr int kSplineLanes = 8, kSplinePostThreads = kSplineLanes * kPostFuse;
__global__ void __launch_bounds__(kSplinePostThreads) k_spline_post(double* __restrict__ coef, int ny, int nx,
                                                                     unsigned long long* clocks) {
    AKB_CHAIN_PRIORITY();
    __shared__ double a[kPostFuse * (kPostFuse + 1)];
    const int64_t total = (int64_t)ny * nx;
    constexpr int pitch = kPostFuse + 1;
    const int tid = threadIdx.x;
    const bool clk = blockIdx.x == 0 && tid == 0;  // workgroup 0's phase clocks (diagnostics)
    if (clk) clocks[0] = wall_clock64();
    double* base = coef + (int64_t)blockIdx.x * total;
    for (int64_t k0 = tid; k0 < total; k0 += 16 * kSplinePostThreads) {  // 16 loads in flight per thread
        double t[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int64_t k = k0 + q * kSplinePostThreads;
            t[q] = k < total ? base[k] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int64_t k = k0 + q * kSplinePostThreads;
            if (k >= total) break;
            const int i = (int)(k / nx), j = (int)(k - (int64_t)i * nx);
            a[i * pitch + j] = t[q];
        }
    }
    __syncthreads();
    if (clk) clocks[1] = wall_clock64();
    constexpr int Q = kSplineLanes, SEG = kPostFuse / kSplineLanes;
    if (tid / Q < nx)  // axis 0: the columns
        spline_line_reg<Q, SEG, pitch>(a + tid / Q, ny, tid % Q, clk ? clocks + 4 : nullptr);
    __syncthreads();
    if (clk) clocks[2] = wall_clock64();
    if (tid / Q < ny) spline_line_reg<Q, SEG, 1>(a + (tid / Q) * pitch, nx, tid % Q);  // axis 1: the rows
    __syncthreads();
    if (clk) clocks[3] = wall_clock64();
    for (int64_t k = tid; k < total; k += kSplinePostThreads) {
        const int i = (int)(k / nx), j = (int)(k - (int64_t)i * nx);
        base[k] = a[i * pitch + j];
    }
}

// the post's map in LDS with one pad word per 128 (element k at k + k / 128): a numpy leaf is 128
// consecutive elements, so the nanmean's lanes - a leaf each - then read distinct banks (without the
// pad every lane of a wave hit the same bank)
__device__ __forceinline__ int64_t post_lds(int64_t k) { return k + (k >> 7); }
struct PostLeaf {  // pw_leaf_lds<true>'s sums over the padded map
    const double* a;
    __device__ double val(int i) const {
        const double x = a[post_lds(i)];
        return x != x ? 0.0 : x;
    }
    __device__ double leaf(int o, int n) const {
        if (n < 8) {
            double res = 0.0;
            for (int i = 0; i < n; ++i) res = res + val(o + i);
            return res;
        }
        double r[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = val(o + j);
        int i = 8;
        for (; i < n - (n % 8); i += 8) {
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] = r[j] + val(o + i + j);
        }
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res = res + val(o + i);
        return res;
    }
};

// PostLeaf::leaf(o, 128): numpy's eight accumulators over a 128-element leaf of the padded map, the
// reads issued 8 at a time (fully unrolled: no loop branch between the batches)
__device__ __noinline__ double post_leaf128(const double* smem, int o) {
    const PostLeaf P{smem};
    double r[8];
#pragma unroll
    for (int blk = 0; blk < 16; ++blk) {
        double t[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) t[q] = P.val(o + 8 * blk + q);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int idx = 8 * blk + q;
            r[idx & 7] = idx < 8 ? t[q] : r[idx & 7] + t[q];
        }
    }
    return ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
}

__global__ void __launch_bounds__(kPostThreads) k_pupil_post(PostArgs a) {
    AKB_CHAIN_PRIORITY();
    __shared__ double smem[kPostLds + kPostLds / 128];  // the map, then matrixWave2 - nanmean (when it fits)
    __shared__ PwTree trees[2];        // the nanmean's pairwise trees (waves 0 and 1)
    __shared__ double bufsum[8];
    __shared__ int firstrow[2];
    __shared__ double red[kPostThreads / 64][kMomMax];
    __shared__ double sys[32];
    __shared__ int sflag;
    // basis5's X (per column) and Y (per row), each division once (the moment passes and the plane
    // subtraction would repeat two divisions per point each)
    __shared__ double bX[kPostBasisMax], bY[kPostBasisMax];
    const int64_t total = (int64_t)a.ny * a.nx;
    const int tid = threadIdx.x, w = tid >> 6;
    double* P = a.params;
    if (tid == 0) a.clocks[0] = wall_clock64();
    const bool tab = a.nx <= kPostBasisMax && a.ny <= kPostBasisMax;
    if (tab) {
        for (int j = tid; j < a.nx; j += kPostThreads) bX[j] = a.nx > 1 ? (2.0 * j - (a.nx - 1)) / (double)(a.nx - 1) : 0.0;
        for (int i = tid; i < a.ny; i += kPostThreads) bY[i] = a.ny > 1 ? (2.0 * i - (a.ny - 1)) / (double)(a.ny - 1) : 0.0;
    }
    // the map into LDS when it fits: every thread's loads in flight at once (the passes below then
    // wait for LDS only)
    const bool in_lds = total <= kPostLds;
    if (in_lds) {
        for (int64_t k0 = 0; k0 < total; k0 += 16 * kPostThreads) {
            double t[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int64_t k = k0 + q * kPostThreads + tid;
                if (k < total) t[q] = a.m[k];
            }
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int64_t k = k0 + q * kPostThreads + tid;
                if (k < total) smem[post_lds(k)] = t[q];
            }
        }
        __syncthreads();
    }
    const double* src = in_lds ? smem : a.m;
    auto L = [&](int64_t k) { return in_lds ? post_lds(k) : k; };  // a map index in src / cm
    if (tid == 0) a.clocks[1] = wall_clock64();
    // np.nanmean: numpy's pairwise sum of the NaN-zeroed map, one wave per 8192-element buffer
    // (waves 0 and 1 alternate over the buffers)
    const int nbuf = (int)((total + 8191) / 8192);
    if (w < 2) {
        for (int b = w; b < nbuf; b += 2) {
            const int64_t b0 = (int64_t)b * 8192;
            const int len = (int)(total - b0 < 8192 ? total - b0 : 8192);
            double v;
            if (in_lds && len == 8192) {
                // a full buffer: numpy's split tree is balanced down to 64 leaves of 128 - a lane's
                // leaf (its 128 reads issued in four batches), then the levels left + right as a
                // butterfly (lane 0 ends with the buffer's sum, in the tree's order)
                v = post_leaf128(smem, (int)b0 + 128 * (tid & 63));
                for (int off = 1; off < 64; off <<= 1) v = v + __shfl_down(v, off);
            } else {
                v = in_lds ? pw_tree_wave_get(trees[w], PostLeaf{smem}, (int)b0, len)
                           : pw_tree_wave<true>(trees[w], src + b0, len);
            }
            if ((tid & 63) == 0) bufsum[b] = v;
            wave_sync();
        }
        if (tid == 0) a.clocks[5] = wall_clock64();  // wave 0's pairwise trees done (diagnostics)
    }
    // the finite count, and the map's range (np.nanmin / np.nanmax: the cone solve's error estimate
    // is held to it, FaithfulPupil)
    double cnt[1] = {0.0};
    double lo = INFINITY, hi = -INFINITY;
    for (int64_t k = tid; k < total; k += kPostThreads) {
        const double v = src[L(k)];
        if (v == v) {
            cnt[0] += 1.0;
            lo = fmin(lo, v);
            hi = fmax(hi, v);
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        lo = fmin(lo, __shfl_down(lo, off));
        hi = fmax(hi, __shfl_down(hi, off));
    }
    __shared__ double ext[kPostThreads / 64][2];
    if ((tid & 63) == 0) {
        ext[w][0] = lo;
        ext[w][1] = hi;
    }
    block_sum<1>(cnt, (double(*)[1])red);
    if (tid == 0) a.clocks[6] = wall_clock64();
    double tot = 0.0;
    for (int b = 0; b < nbuf; ++b) tot = tot + bufsum[b];
    const double mean = tot / cnt[0];
    // matrixWave2 - nanmean, the plane correction's input: in LDS when it fits, else in `corrected`
    double* cm = in_lds ? smem : a.corrected;
    __syncthreads();
    for (int64_t k0 = tid; k0 < total; k0 += 4 * kPostThreads) {  // four reads in flight a round
        double t[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t k = k0 + u * kPostThreads;
            t[u] = k < total ? src[L(k)] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t k = k0 + u * kPostThreads;
            if (k < total) cm[L(k)] = t[u] - mean;
        }
    }
    __syncthreads();
    if (tid == 0) a.clocks[2] = wall_clock64();
    // plane_correction_with_nan_and_outlier_filter: the four moment passes of k_moments
    auto moments = [&](int nb, const double* cf, double thr, int mode, double mu, double (&acc)[kMomMax]) {
#pragma unroll
        for (int q = 0; q < kMomMax; ++q) acc[q] = 0.0;
        double cfr[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
        if (cf)
#pragma unroll
            for (int t = 0; t < 5; ++t) cfr[t] = cf[t];
        // four points a round, their LDS reads (value, basis) issued together before the arithmetic
        // (one LDS latency a round, not one per point); the points in the same order per thread
        constexpr int kR = 4;
        PostIdx ix(tid, a.nx);
        for (int64_t k0 = tid; k0 < total; k0 += kR * kPostThreads) {
            double zr[kR], fr[kR][5];
#pragma unroll
            for (int u = 0; u < kR; ++u) {
                const int64_t k = k0 + u * kPostThreads;
                zr[u] = k < total ? cm[L(k)] : __builtin_nan("");
                basis5_tab(bX, bY, ix.i, ix.j, a.ny, a.nx, fr[u]);
                ix.next();
            }
#pragma unroll
            for (int u = 0; u < kR; ++u) {
            const double z = zr[u];
            if (z != z) continue;
            const double (&f)[5] = fr[u];
            double res = 0.0;
            if (cf || mode > 0) {
                double mm = 0.0;
                for (int t = 0; t < 5; ++t) mm = __builtin_fma(cfr[t], f[t], mm);
                res = z - mm;
                if (mode == 0 && !(fabs(res) < thr)) continue;
            }
            if (mode == 1) {
                acc[0] += res;
                acc[20] += 1.0;
            } else if (mode == 2) {
                const double d = res - mu;
                acc[0] = __builtin_fma(d, d, acc[0]);
                acc[20] += 1.0;
            } else {
#pragma unroll
                for (int r = 0; r < 5; ++r) {
#pragma unroll
                    for (int c = r; c < 5; ++c) {
                        const int q = r * 5 - r * (r - 1) / 2 + (c - r);
                        if (nb == 5 || c < 3) acc[q] = __builtin_fma(f[r], f[c], acc[q]);
                    }
                    if (nb == 5 || r < 3) acc[15 + r] = __builtin_fma(f[r], z, acc[15 + r]);
                }
                acc[20] += 1.0;
            }
            }
        }
        // only the slots the mode fills: 2 (the residual passes), 10 (the plane's 3 x 3), 21
        if (mode > 0) {
            double t[2] = {acc[0], acc[20]};
            block_sum<2>(t, (double(*)[2])red);
            acc[0] = t[0];
            acc[20] = t[1];
        } else if (nb == 3) {
            constexpr int slot[10] = {0, 1, 2, 5, 6, 9, 15, 16, 17, 20};
            double t[10];
#pragma unroll
            for (int q = 0; q < 10; ++q) t[q] = acc[slot[q]];
            block_sum<10>(t, (double(*)[10])red);
#pragma unroll
            for (int q = 0; q < 10; ++q) acc[slot[q]] = t[q];
        } else {
            block_sum<kMomMax>(acc, red);
        }
    };
    // the normal equations of nb terms from the moment slots (pupilmap._normal_solve) into sys[25..]
    auto normal_solve = [&](const double (&mom)[kMomMax], auto nbc, int at) {
        constexpr int nb = decltype(nbc)::value;
        if (tid == 0) {
            double A[nb][nb], b[nb];
#pragma unroll
            for (int r = 0; r < nb; ++r) {
#pragma unroll
                for (int c = 0; c < nb; ++c) {
                    const int lo = r < c ? r : c, hi = r < c ? c : r;
                    A[r][c] = mom[lo * 5 - lo * (lo - 1) / 2 + (hi - lo)];
                }
                b[r] = mom[15 + r];
            }
            if (!solve_small_reg<nb>(A, b)) sflag |= 2;
#pragma unroll
            for (int r = 0; r < nb; ++r) sys[at + r] = b[r];
        }
        __syncthreads();
    };
    if (tid == 0) sflag = 0;
    if (tid < 2) firstrow[tid] = a.ny;  // (the NaN-split pass's minima, after the barriers below)
    double acc[kMomMax];
    moments(5, nullptr, 0.0, 0, 0.0, acc);
    if (tid == 0 && acc[20] < 5) sflag |= 1;  // curve_fit refuses fewer points than parameters
    normal_solve(acc, std::integral_constant<int, 5>{}, 0);  // c1 = sys[0..5)
    if (tid == 0) a.clocks[7] = wall_clock64();  // the first fit solved (diagnostics)
    moments(5, sys, 0.0, 1, 0.0, acc);
    const double n1 = acc[20], mu = acc[0] / acc[20];
    moments(5, sys, 0.0, 2, mu, acc);
    const double thr = a.sigma * sqrt(acc[0] / n1);
    moments(3, sys, thr, 0, 0.0, acc);
    if (tid == 0 && acc[20] < 3) sflag |= 1;
    normal_solve(acc, std::integral_constant<int, 3>{}, 8);  // p2 = sys[8..11)
    if (tid == 0) a.clocks[3] = wall_clock64();
    // corrected = (map - nanmean) - plane, and rotate_with_nan's NaN split of it; psf_calc's rotation
    // estimate (:1122-1132) in the same pass: the first valid row of columns nx / 4 and 3 nx / 4 (every
    // point of those columns tested, the smallest row kept)
    {
        const int c1 = a.nx / 4, c3 = a.nx * 3 / 4;
        PostIdx ix(tid, a.nx);
        for (int64_t k = tid; k < total; k += kPostThreads, ix.next()) {
            double f[5];
            basis5_tab(bX, bY, ix.i, ix.j, a.ny, a.nx, f);
            const double pl = __builtin_fma(sys[10], f[2], __builtin_fma(sys[9], f[1], sys[8] * f[0]));
            const double v = cm[L(k)];
            const bool nan = v != v;
            const double o = nan ? v : v - pl;
            cm[L(k)] = o;
            if (in_lds) a.corrected[k] = o;
            a.coef[k] = nan ? 0.0 : o;
            a.coef[total + k] = nan ? 0.0 : 1.0;
            if (o == o) {
                if (ix.j == c1) atomicMin(&firstrow[0], ix.i);
                if (ix.j == c3) atomicMin(&firstrow[1], ix.i);
            }
        }
    }
    // (an LDS-only barrier: nothing here reads the global stores above, so no wave waits for their
    // acknowledgements as __syncthreads' fence would make it)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (tid == 0) {
        const int c1 = a.nx / 4, c3 = a.nx * 3 / 4;
        const int r1 = firstrow[0], r3 = firstrow[1];
        const double q = (r1 < a.ny && r3 < a.ny) ? (double)(r1 - r3) / (double)(c1 - c3) : __builtin_nan("");
        const double rot = atan(q);
        const double deg = rot * (180.0 / 3.14159265358979323846);
        const double cs = cos_deg(deg), sn = sin_deg(deg);
        const double cy = (a.ny - 1) / 2.0, cx = (a.nx - 1) / 2.0;
        sys[16] = rot;
        sys[17] = deg;
        sys[18] = cs;
        sys[19] = sn;
        sys[20] = cy - (cs * cy + sn * cx);
        sys[21] = cx - (-sn * cy + cs * cx);
    }
    __syncthreads();
    // rotate_with_nan(order 3): the B-spline prefilter (k_spline_post / k_spline_block) and the
    // rotation (k_rotate_post) follow as their own launches
    if (tid == 0) {
        P[0] = mean;
        P[1] = cnt[0];
        for (int q = 0; q < 5; ++q) P[2 + q] = sys[q];
        for (int q = 0; q < 3; ++q) P[7 + q] = sys[8 + q];
        P[10] = thr;
        for (int q = 0; q < 6; ++q) P[11 + q] = sys[16 + q];
        P[17] = (double)sflag;
        double mn = ext[0][0], mx = ext[0][1];
        for (int q = 1; q < kPostThreads / 64; ++q) {
            mn = fmin(mn, ext[q][0]);
            mx = fmax(mx, ext[q][1]);
        }
        P[18] = mn;
        P[19] = mx;
        a.clocks[4] = wall_clock64();
    }
}

// match_legendre_multi (legendre_fit.py:59-92) on an n x n map. Z_k = outer(Py[ny_k], Px[nx_k])
// (the product np.outer forms), then per k: s_k = nansum(Z*Z), Zn = Z / sqrt(s_k),
// c_k = nansum(Zn * data), fit_k = c_k * Zn. This kernel writes the rows that numpy sums (mode 0:
// Z*Z, mode 1: Zn*data) and the fits (mode 2); the sums themselves are akb_pairwise_sum_f64's, in
// numpy's pairwise order, so the coefficients match the reference's bit for bit.
struct LegArgs {
    const double* data;
    int n, K, order;
    const double* px;   // (order, n): P_j(linspace(-1, 1, n)) for the columns
    const double* py;   // (order, n): for the rows
    const int* ord;     // (K, 2): (ny, nx)
    const double* s;    // (K,) nansum(Z*Z)    modes 1, 2
    const double* c;    // (K,) coefficients   mode 2
    int mode;
    double* out;        // (K, n*n)
};

__global__ void __launch_bounds__(kBlock) k_legendre_rows(LegArgs a) {
    const int64_t nn = (int64_t)a.n * a.n, total = nn * a.K;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int k = (int)(t / nn);
        const int64_t p = t - (int64_t)k * nn;
        const int r = (int)(p / a.n), col = (int)(p - (int64_t)r * a.n);
        const int ny = a.ord[2 * k], nx = a.ord[2 * k + 1];
        const double z = a.py[(int64_t)ny * a.n + r] * a.px[(int64_t)nx * a.n + col];
        double v;
        if (a.mode == 0) {
            v = z * z;
        } else {
            const double zn = z / sqrt_cr(a.s[k]);
            v = a.mode == 1 ? zn * a.data[p] : a.c[k] * zn;
        }
        a.out[t] = v;
    }
}

// ---- extract_affine_square_region's warps (AKB_raytrace_20250312.py:1109-1115), both in one pass:
// cv2.warpAffine(nan_to_num(img), M, INTER_LINEAR) and cv2.warpAffine(mask, M, INTER_NEAREST) with
// BORDER_CONSTANT 0, then NaN where the warped mask is 0. iM is M inverted as warpAffine inverts it
// (akb_affine_invert). Source coordinates follow OpenCV's fixed point: the affine terms are scaled
// by 2^10 and rounded to nearest even, INTER_LINEAR keeps 5 fractional bits (32 x 32 weight table,
// weights (1 - f) / f products, exact), INTER_NEAREST rounds at 2^9; the bilinear sum is
// v0 w0 + v1 w1 + v2 w2 + v3 w3 left to right, unfused, as OpenCV's double remap forms it.
__device__ __forceinline__ int cv_round(double v) { return __double2int_rn(v); }
__device__ __forceinline__ int sat_short(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }
__device__ __forceinline__ double nan_to_num(double v) {
    if (v != v) return 0.0;
    if (v == INFINITY) return 1.7976931348623157e308;
    if (v == -INFINITY) return -1.7976931348623157e308;
    return v;
}

struct WarpArgs {
    const double* img;
    int ny, nx;
    double m0, m1, m2, m3, m4, m5;  // the inverse map: source = (m0 x + m1 y + m2, m3 x + m4 y + m5)
    int side;
    double* out;
};

__global__ void __launch_bounds__(256) k_warp_affine(WarpArgs a) {
    const int64_t n = (int64_t)a.side * a.side;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(i / a.side), x = (int)(i - (int64_t)y * a.side);
        const int xr = cv_round((a.m1 * y + a.m2) * 1024);
        const int yr = cv_round((a.m4 * y + a.m5) * 1024);
        const int adelta = cv_round(a.m0 * x * 1024), bdelta = cv_round(a.m3 * x * 1024);
        // INTER_NEAREST mask
        const int xn = sat_short((xr + 512 + adelta) >> 10), yn = sat_short((yr + 512 + bdelta) >> 10);
        bool valid = false;
        if ((unsigned)xn < (unsigned)a.nx && (unsigned)yn < (unsigned)a.ny) {
            const double v = a.img[(int64_t)yn * a.nx + xn];
            valid = v == v;
        }
        if (!valid) {
            a.out[i] = NAN;
            continue;
        }
        // INTER_LINEAR value
        const int X = (xr + 16 + adelta) >> 5, Y = (yr + 16 + bdelta) >> 5;
        const int sx = sat_short(X >> 5), sy = sat_short(Y >> 5);
        const int fx = X & 31, fy = Y & 31;
        const double ax = fx * (1.0 / 32), ay = fy * (1.0 / 32);
        const double w0 = (1.0 - ay) * (1.0 - ax), w1 = (1.0 - ay) * ax, w2 = ay * (1.0 - ax), w3 = ay * ax;
        double v0, v1, v2, v3;
        if ((unsigned)sx < (unsigned)(a.nx - 1) && (unsigned)sy < (unsigned)(a.ny - 1)) {
            const double* s = a.img + (int64_t)sy * a.nx + sx;
            v0 = nan_to_num(s[0]);
            v1 = nan_to_num(s[1]);
            v2 = nan_to_num(s[a.nx]);
            v3 = nan_to_num(s[a.nx + 1]);
        } else if (sx >= a.nx || sx + 1 < 0 || sy >= a.ny || sy + 1 < 0) {
            a.out[i] = 0.0;
            continue;
        } else {
            const int x0 = sx >= 0 && sx < a.nx ? sx : -1, x1 = sx + 1 >= 0 && sx + 1 < a.nx ? sx + 1 : -1;
            const int y0 = sy >= 0 && sy < a.ny ? sy : -1, y1 = sy + 1 >= 0 && sy + 1 < a.ny ? sy + 1 : -1;
            v0 = x0 >= 0 && y0 >= 0 ? nan_to_num(a.img[(int64_t)y0 * a.nx + x0]) : 0.0;
            v1 = x1 >= 0 && y0 >= 0 ? nan_to_num(a.img[(int64_t)y0 * a.nx + x1]) : 0.0;
            v2 = x0 >= 0 && y1 >= 0 ? nan_to_num(a.img[(int64_t)y1 * a.nx + x0]) : 0.0;
            v3 = x1 >= 0 && y1 >= 0 ? nan_to_num(a.img[(int64_t)y1 * a.nx + x1]) : 0.0;
        }
        a.out[i] = v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3;
    }
}

// mask = 255 where img is not NaN (extract_affine_square_region's valid_mask_uint8, :1063-1064)
__global__ void __launch_bounds__(256) k_valid_mask(const double* __restrict__ img, int64_t n, uint8_t* __restrict__ m) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double v = img[i];
        m[i] = v == v ? 255 : 0;
    }
}

}  // namespace akb

using namespace akb;

extern "C" {

int akb_first_valid_rows_f64(const double* m, int ny, int nx, int32_t* d_rows, void* stream) {
    clear_error();
    AKB_REQUIRE(m && d_rows && ny > 0 && nx > 0, "bad arguments");
    k_first_valid_rows<<<(nx + kBlock - 1) / kBlock, kBlock, 0, (hipStream_t)stream>>>(m, ny, nx, d_rows);
    return launch_status("k_first_valid_rows");
}

int64_t akb_rotate_work_bytes(int ny, int nx) { return (ny > 0 && nx > 0) ? (int64_t)2 * ny * nx * 8 : -1; }

int akb_rotate_with_nan_f64(const double* m, int ny, int nx, const double rot[4], const double offset[2],
                            double* rotated, double* opd_m, void* work, void* stream) {
    clear_error();
    AKB_REQUIRE(m && rot && offset && rotated && work && ny > 0 && nx > 0, "bad arguments");
    hipStream_t s = (hipStream_t)stream;
    double* coef = (double*)work;
    const int64_t n = (int64_t)ny * nx;
    k_nan_split<<<grid_for(n), kBlock, 0, s>>>(m, n, coef);
    int st = launch_status("k_nan_split");
    if (st) return st;
    k_spline_lines<<<dim3((nx + 63) / 64, 2), 64, 0, s>>>(coef, ny, nx, 0);
    if ((st = launch_status("k_spline_lines(axis 0)"))) return st;
    k_spline_lines<<<dim3((ny + 63) / 64, 2), 64, 0, s>>>(coef, ny, nx, 1);
    if ((st = launch_status("k_spline_lines(axis 1)"))) return st;
    RotArgs a{coef, ny, nx, rot[0], rot[1], rot[2], rot[3], offset[0], offset[1], rotated, opd_m};
    k_rotate_cubic<<<grid_for(n), kBlock, 0, s>>>(a);
    return launch_status("k_rotate_cubic");
}

int64_t akb_moments_work_bytes(void) { return (int64_t)(512 * kMomMax + kMomMax) * 8; }

int akb_map_moments_f64(const double* z, int ny, int nx, int nb, const double* d_coef, double thr, int mode,
                        double mean, double* d_out, void* work, void* stream) {
    clear_error();
    AKB_REQUIRE(z && d_out && work && ny > 0 && nx > 0, "bad arguments");
    AKB_REQUIRE(nb == 3 || nb == 5, "basis of 3 or 5 terms");
    AKB_REQUIRE(mode >= 0 && mode <= 2 && (mode == 0 || d_coef), "bad mode");
    hipStream_t s = (hipStream_t)stream;
    MomArgs a{z, ny, nx, nb, d_coef, thr, mode, mean, (double*)work};
    const int64_t n = (int64_t)ny * nx;
    const unsigned g = grid_for(n, 4) < 512 ? grid_for(n, 4) : 512;
    k_moments<<<g, kBlock, 0, s>>>(a);
    int st = launch_status("k_moments");
    if (st) return st;
    k_moments_final<<<1, 64, 0, s>>>((double*)work, (int)g, d_out);
    return launch_status("k_moments_final");
}

int akb_plane_subtract_f64(const double* z, int ny, int nx, const double* d_coef3, double* out, void* stream) {
    clear_error();
    AKB_REQUIRE(z && d_coef3 && out && ny > 0 && nx > 0, "bad arguments");
    k_plane_subtract<<<grid_for((int64_t)ny * nx), kBlock, 0, (hipStream_t)stream>>>(z, ny, nx, d_coef3, out);
    return launch_status("k_plane_subtract");
}

// the post's work: phase clocks (16 words) | coef (2 ny nx)
constexpr int64_t kPostHead = 16;
int64_t akb_pupil_post_work_bytes(int ny, int nx) {
    if (ny < 1 || nx < 1) return -1;
    return (kPostHead + 2 * (int64_t)ny * nx) * 8;
}

int akb_pupil_post_f64(const double* map, int ny, int nx, double sigma, double* corrected, double* rotated,
                       double* opd, void* work, double* d_params, void* stream) {
    clear_error();
    AKB_REQUIRE(map && corrected && rotated && opd && work && d_params && ny > 1 && nx > 1, "bad arguments");
    AKB_REQUIRE((int64_t)ny * nx <= kPostMax, "the post handles maps of up to 65536 points");
    hipStream_t s = (hipStream_t)stream;
    const int64_t total = (int64_t)ny * nx;
    double* const head = (double*)work;
    double* const w = head + kPostHead;  // coef
    PostArgs a{map, ny, nx, sigma, corrected, w, d_params, (unsigned long long*)head};
    k_pupil_post<<<1, kPostThreads, 0, s>>>(a);
    int st = launch_status("k_pupil_post");
    if (st) return st;
    if (ny <= kPostFuse && nx <= kPostFuse) {
        k_spline_post<<<2, kSplinePostThreads, 0, s>>>(w, ny, nx, (unsigned long long*)head + 8);
        if ((st = launch_status("k_spline_post"))) return st;
    } else {
        for (int axis = 0; axis < 2; ++axis) {
            const int nlines = axis == 0 ? nx : ny, len = axis == 0 ? ny : nx;
            if (len <= kSplineMaxLen)
                k_spline_block<<<dim3((nlines + kSplineLines - 1) / kSplineLines, 2), kSplineThreads, 0, s>>>(w, ny, nx,
                                                                                                            axis);
            else
                k_spline_lines<<<dim3((nlines + 63) / 64, 2), 64, 0, s>>>(w, ny, nx, axis);
            if ((st = launch_status("k_spline"))) return st;
        }
    }
    k_rotate_post<<<grid_for(total, 4, 128), kBlock, 0, s>>>(w, ny, nx, d_params, rotated, opd);
    return launch_status("k_rotate_post");
}

int akb_legendre_rows_f64(const double* data, int n, int K, int order, const double* px, const double* py,
                          const int* ord, const double* s, const double* c, int mode, double* out, void* stream) {
    clear_error();
    AKB_REQUIRE(n > 0 && K > 0 && order > 0 && px && py && ord && out, "bad arguments");
    AKB_REQUIRE(mode >= 0 && mode <= 2, "mode 0, 1 or 2");
    AKB_REQUIRE(mode == 0 || s, "mode 1 / 2 need the norms");
    AKB_REQUIRE(mode != 1 || data, "mode 1 needs the map");
    AKB_REQUIRE(mode != 2 || c, "mode 2 needs the coefficients");
    LegArgs a{data, n, K, order, px, py, ord, s, c, mode, out};
    k_legendre_rows<<<grid_for((int64_t)n * n * K), kBlock, 0, (hipStream_t)stream>>>(a);
    return launch_status("k_legendre_rows");
}

int akb_valid_mask_u8(const double* img, int ny, int nx, uint8_t* mask, void* stream) {
    AKB_REQUIRE(img && mask && ny > 0 && nx > 0, "arguments");
    const int64_t n = (int64_t)ny * nx;
    akb::k_valid_mask<<<akb::grid_for(n, 4), 256, 0, (hipStream_t)stream>>>(img, n, mask);
    return akb::launch_status("k_valid_mask");
}

int akb_warp_affine_f64(const double* img, int ny, int nx, const double* iM, int side, double* out, void* stream) {
    AKB_REQUIRE(img && iM && out && ny > 0 && nx > 0 && side > 0, "arguments");
    akb::WarpArgs a{img, ny, nx, iM[0], iM[1], iM[2], iM[3], iM[4], iM[5], side, out};
    const int64_t n = (int64_t)side * side;
    akb::k_warp_affine<<<akb::grid_for(n, 4), 256, 0, (hipStream_t)stream>>>(a);
    return akb::launch_status("k_warp_affine");
}

}  // extern "C"

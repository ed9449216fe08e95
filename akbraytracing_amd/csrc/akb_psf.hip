// Fraunhofer PSF by FFT for gfx950: compute_psf_fft (psf_fft.py:29-125) as
//   k_psf_pupil  : NaN mask -> U = A exp(i 2pi/lambda opd) -> optional Hann -> even-size pad ->
//                  centred zero-pad x pad_factor -> ifftshift, all folded into one index map that
//                  writes the FFT input directly (one pass, complex128, batch = wavelengths)
//   rocFFT       : in-place 2-D complex-to-complex forward transform, batched over wavelengths
//   k_psf_inten  : fftshift folded into the read index, * dA, |U|^2 -> psf, per-wavelength max
//   k_psf_norm   : psf /= Imax (and efield / sqrt(Imax))
// The transform is HBM-bound (a 2048^2 complex128 plane is 64 MiB); the pre/post kernels are
// single streaming passes.
#include <math.h>
#include <string.h>
#include <rocfft/rocfft.h>

#include <map>
#include <mutex>
#include <tuple>
#include <type_traits>

#include "akb_common.h"

namespace akb {

struct PsfGeom {
    int ny, nx;        // pupil
    int ny2, nx2;      // after ensure_even_size
    int py, px;        // padded
    int pad_y0, pad_x0;
};

static PsfGeom psf_geom(int ny, int nx, int pad) {
    PsfGeom g;
    g.ny = ny;
    g.nx = nx;
    g.ny2 = ny + (ny % 2);
    g.nx2 = nx + (nx % 2);
    g.py = g.ny2 * pad;
    g.px = g.nx2 * pad;
    g.pad_y0 = (g.py - g.ny2) / 2;
    g.pad_x0 = (g.px - g.nx2) / 2;
    return g;
}

struct PsfPupilArgs {
    const double* opd;
    const double* amp;
    const double* wy;
    const double* wx;
    double wmax;
    PsfGeom g;
    double kphase[8];  // 2*pi/lambda per batch entry (host-computed like numpy's scalar)
    double2* field;
};

// writes ifftshift(pad(U)) for batch entry blockIdx.z
__global__ void __launch_bounds__(kBlock) k_psf_pupil(PsfPupilArgs a) {
    const PsfGeom g = a.g;
    const int b = blockIdx.z;
    const double kp = a.kphase[b];
    double2* F = a.field + (int64_t)b * g.py * g.px;
    const int hy = g.py / 2, hx = g.px / 2;
    for (int yo = blockIdx.y; yo < g.py; yo += gridDim.y)
    for (int xo = blockIdx.x * blockDim.x + threadIdx.x; xo < g.px; xo += gridDim.x * blockDim.x) {
        // ifftshift for even lengths: out[i] = in[(i + n/2) % n]
        int ys = yo + hy;
        if (ys >= g.py) ys -= g.py;
        int xs = xo + hx;
        if (xs >= g.px) xs -= g.px;
        const int yy = ys - g.pad_y0;
        const int xx = xs - g.pad_x0;
        double re = 0.0, im = 0.0;
        if (yy >= 0 && yy < g.ny && xx >= 0 && xx < g.nx) {
            const int64_t pi = (int64_t)yy * g.nx + xx;
            double o = a.opd[pi];
            // amp == NULL: psf_calc's mask, 1 where the OPD is defined and 0 elsewhere (:1182-1188)
            double A = a.amp ? a.amp[pi] : (isfinite(o) ? 1.0 : 0.0);
            if (!isfinite(A)) A = 0.0;
            if (!isfinite(o)) o = 0.0;
            const double ph = kp * o;
            double s, c;
            sincos(ph, &s, &c);
            // A * exp(i ph) as numpy: (A*c - 0*s, A*s + 0*c)
            re = A * c - 0.0 * s;
            im = A * s + 0.0 * c;
            if (a.wy) {
                const double w = (a.wy[yy] * a.wx[xx]) / a.wmax;
                const double r0 = re, i0 = im;
                re = r0 * w - i0 * 0.0;
                im = r0 * 0.0 + i0 * w;
            }
        }
        F[(int64_t)yo * g.px + xo] = make_double2(re, im);
    }
}

__device__ __forceinline__ void atomic_max_nonneg(double* addr, double v) {
    // non-negative doubles order like their bit patterns; NaN (0x7ff8...) orders above +inf,
    // which reproduces numpy's NaN-propagating max. Thousands of workgroups meet on one word:
    // only those holding a new maximum issue the atomic (a handful), the rest read and skip.
    unsigned long long* a = (unsigned long long*)addr;
    const unsigned long long k = (unsigned long long)__double_as_longlong(v);
    if (k > __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(a, k);
}

struct PsfIntenArgs {
    const double2* field;
    PsfGeom g;
    double dA;
    const double* pitch;  // device [dx, dy] or NULL
    double* psf;
    double2* efield;
    double* imax;
};

__global__ void __launch_bounds__(kBlock) k_psf_inten(PsfIntenArgs a) {
    const PsfGeom g = a.g;
    const int b = blockIdx.z;
    const int64_t total = (int64_t)g.py * g.px;
    const double2* F = a.field + (int64_t)b * total;
    double* P = a.psf + (int64_t)b * total;
    double2* E = a.efield ? a.efield + (int64_t)b * total : nullptr;
    const int hy = g.py / 2, hx = g.px / 2;
    const double dA = a.pitch ? a.pitch[0] * a.pitch[1] : a.dA;
    double m = 0.0;
    for (int yo = blockIdx.y; yo < g.py; yo += gridDim.y)
    for (int xo = blockIdx.x * blockDim.x + threadIdx.x; xo < g.px; xo += gridDim.x * blockDim.x) {
        const int64_t idx = (int64_t)yo * g.px + xo;
        int ys = yo + hy;
        if (ys >= g.py) ys -= g.py;
        int xs = xo + hx;
        if (xs >= g.px) xs -= g.px;
        const double2 f = F[(int64_t)ys * g.px + xs];
        // U_im = fftshift(F) * dA (complex * real as numpy)
        const double re = f.x * dA - f.y * 0.0;
        const double im = f.x * 0.0 + f.y * dA;
        const double h = hypot(re, im);
        const double I = h * h;
        P[idx] = I;
        if (E) E[idx] = make_double2(re, im);
        m = (I > m || I != I) ? I : m;
    }
    // wave max, then workgroup max through LDS, then one atomic per workgroup (a per-wave
    // atomic on one word serialises ~65k atomics for a 2048^2 plane)
    __shared__ double wmax[kBlock / 64];
    for (int off = 32; off > 0; off >>= 1) {
        const double o = __shfl_down(m, off);
        m = (o > m || o != o) ? o : m;
    }
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / 64; ++w) m = (wmax[w] > m || wmax[w] != wmax[w]) ? wmax[w] : m;
        atomic_max_nonneg(a.imax + b, m);
    }
}

__global__ void __launch_bounds__(kBlock) k_psf_norm(double* psf, double2* efield, const double* imax,
                                                     int64_t total) {
    const int b = blockIdx.z;
    const double im = imax[b];
    const bool pos = im > 0.0;
    const double sq = sqrt(pos ? im : 1.0);
    double* P = psf + (int64_t)b * total;
    double2* E = efield ? efield + (int64_t)b * total : nullptr;
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        if (pos) P[idx] = P[idx] / im;
        if (E) {
            const double2 e = E[idx];
            E[idx] = make_double2(e.x / sq, e.y / sq);
        }
    }
}

// ---- pruned transform: the padded plane is never built ----
//
// The padded field is zero outside the ey x ex pupil block, so with centred indices
// a' = a - ey/2, b' = b - ex/2 and output indices ko, lo of the fftshift-ed plane
//   F[ko][lo] = (-1)^((ey+ex)/2) e^{i pi ko/pad} e^{i pi lo/pad}
//               * sum_a (-1)^a sum_b (-1)^b U0[a][b] W_px^(lo b) W_py^(ko a)
// and with lo = pad j + r the inner sum is an ex-point DFT of U0[a][b] (-1)^b W_px^(r b) at j
// (likewise for the columns). Rows pass: ey x pad FFTs of length ex -> H (ey x px, 4 MiB for a
// 128^2 pupil at pad 16); column pass: px x pad FFTs of length ey, straight to |F dA|^2. The
// column pass runs twice (peak, then the normalised write) instead of writing the unnormalised
// plane and re-reading it: the only HBM traffic is the output itself. Each FFT is a four-step
// split N = N1 N2 into in-register DFTs and one LDS exchange, twiddles of the pad split from a
// W_P table in device memory.
// Taken when ey and ex are powers of two in [8, 256]; rocFFT on the full plane otherwise.
constexpr int kFftTile = 2048;  // complex points per workgroup

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

__global__ void __launch_bounds__(kBlock) k_psf_twiddle(double2* W, int P) {
    AKB_CHAIN_PRIORITY();
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < P; t += gridDim.x * blockDim.x) {
        double sn, cs;
        sincospi(2.0 * (double)t / (double)P, &sn, &cs);
        W[t] = make_double2(cs, -sn);  // exp(-2 pi i t / P)
    }
}

// exp(-2 pi i k / 32), k < 16 (W_M^k = W_32^(k 32 / M) for M <= 32)
constexpr double kW32re[16] = {0x1.0000000000000p+0,  0x1.f6297cff75cb0p-1,  0x1.d906bcf328d46p-1,
                               0x1.a9b66290ea1a3p-1,  0x1.6a09e667f3bcdp-1,  0x1.1c73b39ae68c8p-1,
                               0x1.87de2a6aea963p-2,  0x1.8f8b83c69a60bp-3,  0.0,
                               -0x1.8f8b83c69a60bp-3, -0x1.87de2a6aea963p-2, -0x1.1c73b39ae68c8p-1,
                               -0x1.6a09e667f3bcdp-1, -0x1.a9b66290ea1a3p-1, -0x1.d906bcf328d46p-1,
                               -0x1.f6297cff75cb0p-1};
constexpr double kW32im[16] = {0.0,                   -0x1.8f8b83c69a60bp-3, -0x1.87de2a6aea963p-2,
                               -0x1.1c73b39ae68c8p-1, -0x1.6a09e667f3bcdp-1, -0x1.a9b66290ea1a3p-1,
                               -0x1.d906bcf328d46p-1, -0x1.f6297cff75cb0p-1, -0x1.0000000000000p+0,
                               -0x1.f6297cff75cb0p-1, -0x1.d906bcf328d46p-1, -0x1.a9b66290ea1a3p-1,
                               -0x1.6a09e667f3bcdp-1, -0x1.1c73b39ae68c8p-1, -0x1.87de2a6aea963p-2,
                               -0x1.8f8b83c69a60bp-3};

constexpr int ilog2_c(int m) { return m <= 1 ? 0 : 1 + ilog2_c(m / 2); }
constexpr int bitrev_c(int i, int bits) {
    int r = 0;
    for (int k = 0; k < bits; ++k) r |= ((i >> k) & 1) << (bits - 1 - k);
    return r;
}

// in-register DFT of size M (power of two <= 32): v holds x[bitrev(i)] at i on entry (the caller
// loads in that order) and X[k] at k on exit; radix-2 DIT, every index and twiddle resolved at
// compile time, in place
// a * b with fused multiply-adds (the line transforms: their bar is 1e-10 of the peak, not bits)
__device__ __forceinline__ double2 cmulf(double2 a, double2 b) {
    return make_double2(fma(a.x, b.x, -(a.y * b.y)), fma(a.x, b.y, a.y * b.x));
}

template <int M, bool kFma = false>
__device__ __forceinline__ void dft_reg_br(double2 (&t)[M]) {
#pragma unroll
    for (int h = 1; h < M; h <<= 1) {  // half-length of the current butterflies
#pragma unroll
        for (int i = 0; i < M; i += 2 * h) {
#pragma unroll
            for (int k = 0; k < h; ++k) {
                const double2 x = t[i + k];
                double2 y = t[i + k + h];
                if (k != 0) {
                    if (2 * k == h) {
                        y = make_double2(y.y, -y.x);  // * W^(len/4) = -i
                    } else {
                        const int wi = k * (16 / h);
                        const double2 w = make_double2(kW32re[wi], kW32im[wi]);
                        y = kFma ? cmulf(y, w) : cmul(y, w);
                    }
                }
                t[i + k] = make_double2(x.x + y.x, x.y + y.y);
                t[i + k + h] = make_double2(x.x - y.x, x.y - y.y);
            }
        }
    }
}

// C transforms of length N = N1 N2 per workgroup (C * N2 threads, column c fastest):
//   step 1: thread (c, n2) takes x[n1 N2 + n2], n1 < N1, an N1-point DFT in registers, twiddle
//           W_N^(n2 k1); LDS exchange
//   step 2: thread (c, t2) runs the N2-point DFTs of k1 = t2 + s N2, giving X[k1 + N1 k2]
// load(c, a) supplies input element a of transform c; store(c, j, value) consumes output j.
// N <= 256: two stages (N1 x N2, N1 <= 16 complex values per thread). N = 512 / 1024: three
// stages (fft_block3: NA = 8 / 16 in registers, then the remaining 64-point transforms as 8 x 8),
// so no thread holds more than 16 complex values - a 32-point register DFT needs ~290 VGPRs and
// runs one wave per SIMD.
template <int N>
struct FftShape {
    static constexpr int L = ilog2_c(N);
    static constexpr bool k3 = N >= 512;
    static constexpr int NA = N >= 1024 ? 16 : 8;  // first stage of the three-stage split
    static constexpr int N1 = k3 ? NA : 1 << ((L + 1) / 2);
    static constexpr int N2 = N / N1;  // threads per transform (both splits)
    static constexpr int C0 = kFftTile / N < kBlock / N2 ? kFftTile / N : kBlock / N2;
};

// three stages for N = NA * M, M = 64 = 8 x 8: stage A, thread (c, m) takes x[nA M + m], an
// NA-point DFT, twiddle W_N^(m kA) -> Y[kA][m]; stage B1, for each kA the 64-point transform's
// first 8-point DFTs over m = mb1 8 + mb2 (in place in Y[kA], twiddle W_64^(mb2 kb1)); stage B2,
// the second 8-point DFTs give Z_kA[kb1 + 8 kb2] = X[kA + NA (kb1 + 8 kb2)].
template <int N, typename Load, typename Store>
__device__ __forceinline__ void fft_block3(int C, double2* Y, const double2* twN, Load load, Store store) {
    constexpr int NA = FftShape<N>::NA, M = N / NA, MB = 8;
    static_assert(M == MB * MB, "three-stage split: N / NA must be 64");
    constexpr int LA = ilog2_c(NA), LB = ilog2_c(MB);
    const int tid = threadIdx.x;
    const int c = tid % C, p = tid / C;  // p < M: this thread's task in each stage
    {
        const int m = p;
        double2 v[NA];
#pragma unroll
        for (int i = 0; i < NA; ++i) v[i] = load(c, bitrev_c(i, LA) * M + m);
        dft_reg_br<NA>(v);
#pragma unroll
        for (int kA = 0; kA < NA; ++kA) {
            const double2 w = kA && m ? cmul(v[kA], twN[(m * kA) % N]) : v[kA];
            Y[(kA * M + m) * C + c] = w;
        }
    }
    __syncthreads();
    // stage B1: NA * 8 tasks (kA, mb2) over M threads
#pragma unroll
    for (int s = 0; s < NA * MB / M; ++s) {
        const int task = p + s * M;
        const int kA = task / MB, mb2 = task % MB;
        double2 w[MB];
#pragma unroll
        for (int i = 0; i < MB; ++i) w[i] = Y[(kA * M + bitrev_c(i, LB) * MB + mb2) * C + c];
        dft_reg_br<MB>(w);
#pragma unroll
        for (int kb1 = 0; kb1 < MB; ++kb1) {
            const double2 t = kb1 && mb2 ? cmul(w[kb1], twN[(NA * mb2 * kb1) % N]) : w[kb1];
            Y[(kA * M + kb1 * MB + mb2) * C + c] = t;
        }
    }
    __syncthreads();
    // stage B2: NA * 8 tasks (kA, kb1)
#pragma unroll
    for (int s = 0; s < NA * MB / M; ++s) {
        const int task = p + s * M;
        const int kA = task / MB, kb1 = task % MB;
        double2 u[MB];
#pragma unroll
        for (int i = 0; i < MB; ++i) u[i] = Y[(kA * M + kb1 * MB + bitrev_c(i, LB)) * C + c];
        dft_reg_br<MB>(u);
#pragma unroll
        for (int kb2 = 0; kb2 < MB; ++kb2) store(c, kA + NA * (kb1 + MB * kb2), u[kb2]);
    }
}

template <int N, typename Load, typename Store>
__device__ __forceinline__ void fft_block2(int C, double2* Y, const double2* twN, Load load, Store store) {
    constexpr int N1 = FftShape<N>::N1, N2 = FftShape<N>::N2;
    constexpr int L1 = ilog2_c(N1), L2 = ilog2_c(N2);
    const int tid = threadIdx.x;
    const int c = tid % C, n2 = tid / C;
    {
        double2 v[N1];
#pragma unroll
        for (int i = 0; i < N1; ++i) v[i] = load(c, bitrev_c(i, L1) * N2 + n2);
        dft_reg_br<N1>(v);
#pragma unroll
        for (int k1 = 0; k1 < N1; ++k1) {
            const double2 w = k1 && n2 ? cmul(v[k1], twN[(n2 * k1) % N]) : v[k1];
            Y[(k1 * N2 + n2) * C + c] = w;
        }
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < N1 / N2; ++s) {
        const int k1 = n2 + s * N2;
        double2 w[N2];
#pragma unroll
        for (int i = 0; i < N2; ++i) w[i] = Y[(k1 * N2 + bitrev_c(i, L2)) * C + c];
        dft_reg_br<N2>(w);
#pragma unroll
        for (int k2 = 0; k2 < N2; ++k2) store(c, k1 + N1 * k2, w[k2]);
    }
}

template <int N, typename Load, typename Store>
__device__ __forceinline__ void fft_block(int C, double2* Y, const double2* twN, Load load, Store store) {
    if constexpr (FftShape<N>::k3)
        fft_block3<N>(C, Y, twN, load, store);
    else
        fft_block2<N>(C, Y, twN, load, store);
}

struct PsfFastArgs {
    const double* opd;
    const double* amp;
    const double* wy;
    const double* wx;
    double wmax;
    PsfGeom g;
    double kphase[8];
    const double2* Wx;  // W_px table
    const double2* Wy;  // W_py table
    double2* H;         // (batch, ey, px), or (batch, px, ey) when hT (column length >= 512)
    int hT;
    double dA;
    const double* pitch;
    double* psf;
    double2* efield;
    double* imax;
};

// row pass: workgroup (row a, chunk of r, batch) -> H[b][a][pad j + r], N = ex
template <int N>
__global__ void __launch_bounds__(kBlock) k_psf_rows(PsfFastArgs A) {
    constexpr int C0 = FftShape<N>::C0;
    __shared__ double2 Y[C0 * N];
    __shared__ double2 u[N];
    __shared__ double2 tw[N];
    const PsfGeom g = A.g;
    const int a = blockIdx.x, b = blockIdx.z;
    const int pad = g.px / N;
    const int r0 = blockIdx.y * C0;
    if (a == 0 && blockIdx.y == 0 && threadIdx.x == 0) A.imax[b] = 0.0;  // column passes follow
    for (int m = threadIdx.x; m < N; m += blockDim.x) {
        tw[m] = A.Wx[(int64_t)m * pad];
        // pupil row a with (-1)^col folded in (rows / cols past ny, nx: the even-size zero pad)
        double re = 0.0, im = 0.0;
        if (a < g.ny && m < g.nx) {
            const int64_t pi = (int64_t)a * g.nx + m;
            double o = A.opd[pi];
            double amp = A.amp ? A.amp[pi] : (isfinite(o) ? 1.0 : 0.0);
            if (!isfinite(amp)) amp = 0.0;
            if (!isfinite(o)) o = 0.0;
            double sn, cs;
            sincos(A.kphase[b] * o, &sn, &cs);
            re = amp * cs - 0.0 * sn;
            im = amp * sn + 0.0 * cs;
            if (A.wy) {
                const double w = (A.wy[a] * A.wx[m]) / A.wmax;
                const double x0 = re, y0 = im;
                re = x0 * w - y0 * 0.0;
                im = x0 * 0.0 + y0 * w;
            }
        }
        if (m & 1) {
            re = -re;
            im = -im;
        }
        u[m] = make_double2(re, im);
    }
    __syncthreads();
    double2* Hrow = A.H + ((int64_t)b * g.ny2 + a) * g.px;
    // transposed H for long columns: the column pass then reads each column contiguously (its
    // 32 reads of H are what the scattered write here pays for once)
    double2* Ht = A.H + (int64_t)b * g.ny2 * g.px + a;
    fft_block<N>(
        C0, Y, tw,
        [&](int c, int m) {
            const int r = r0 + c;
            return r < pad ? cmul(u[m], A.Wx[r * m]) : make_double2(0.0, 0.0);
        },
        [&](int c, int j, double2 v) {
            const int r = r0 + c;
            if (r < pad) {
                if (A.hT)
                    Ht[((int64_t)pad * j + r) * g.ny2] = v;
                else
                    Hrow[(int64_t)pad * j + r] = v;
            }
        });
}

__device__ __forceinline__ double dmax_nan(double m, double v) { return (v > m || v != v) ? v : m; }

// column pass: workgroup (column tile, r, batch), N = ey; kWrite = false: the peak only;
// true: normalised intensity (and efield) at rows ko = pad j + r of the tile's columns
template <int N, bool kWrite>
__global__ void __launch_bounds__(kBlock) k_psf_cols(PsfFastArgs A, int C) {
    constexpr int C0 = FftShape<N>::C0;
    __shared__ double2 Y[C0 * N];
    __shared__ double2 tw[N];
    __shared__ double2 twr[N];  // (-1)^a W_py^(r a), the input twiddle of this workgroup's r
    __shared__ double wm[kBlock / 64];
    const PsfGeom g = A.g;
    const int pad = g.py / N;
    const int l0 = blockIdx.x * C, r = blockIdx.y, b = blockIdx.z;
    for (int m = threadIdx.x; m < N; m += blockDim.x) {
        tw[m] = A.Wy[(int64_t)m * pad];
        const double2 w = A.Wy[r * m];
        twr[m] = (m & 1) ? make_double2(-w.x, -w.y) : w;
    }
    __syncthreads();
    const double2* Hb = A.H + (int64_t)b * N * g.px;
    const double dA = A.pitch ? A.pitch[0] * A.pitch[1] : A.dA;
    const double sgn = ((N / 2 + g.nx2 / 2) & 1) ? -1.0 : 1.0;
    // |F dA|^2 does not need the unit-modulus phase factors: the peak and the write pass both
    // take it from the raw transform; only the efield gets the phases and the sign
    double scale = 1.0, sq = 1.0;
    if (kWrite) {
        const double imx = A.imax[b];
        scale = imx > 0.0 ? 1.0 / imx : 1.0;
        sq = sqrt(imx > 0.0 ? imx : 1.0);
    }
    double* P = A.psf + (int64_t)b * g.py * g.px;
    double2* E = A.efield ? A.efield + (int64_t)b * g.py * g.px : nullptr;
    double m = 0.0;
    fft_block<N>(
        C, Y, tw,
        [&](int c, int a) {
            const int64_t h = FftShape<N>::k3 ? (int64_t)(l0 + c) * N + a : (int64_t)a * g.px + l0 + c;
            return cmul(Hb[h], twr[a]);
        },
        [&](int c, int j, double2 f) {
            const int ko = pad * j + r, lo = l0 + c;
            const double re = f.x * dA, im = f.y * dA;
            const double I = re * re + im * im;
            if (kWrite) {
                const int64_t idx = (int64_t)ko * g.px + lo;
                P[idx] = I * scale;
                if (E) {
                    // e^{i pi ko / pad} = conj(W_py^(ko ey / 2)), likewise for lo; then the sign
                    const double2 py_ph = A.Wy[((int64_t)ko * (N / 2)) % g.py];
                    const double2 px_ph = A.Wx[((int64_t)lo * (g.nx2 / 2)) % g.px];
                    double2 e = cmul(make_double2(re, im), make_double2(py_ph.x, -py_ph.y));
                    e = cmul(e, make_double2(px_ph.x, -px_ph.y));
                    E[idx] = make_double2(sgn * e.x / sq, sgn * e.y / sq);
                }
            } else {
                m = dmax_nan(m, I);
            }
        });
    if (!kWrite) {
        for (int off = 32; off > 0; off >>= 1) m = dmax_nan(m, __shfl_down(m, off));
        if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int w = 1; w < (int)(blockDim.x + 63) / 64; ++w) m = dmax_nan(m, wm[w]);
            atomic_max_nonneg(A.imax + b, m);
        }
    }
}

template <int N>
static int launch_psf_rows(const PsfFastArgs& fa, int batch, hipStream_t s) {
    constexpr int C0 = FftShape<N>::C0;
    const int pad = fa.g.px / N;
    k_psf_rows<N><<<dim3(fa.g.ny2, (pad + C0 - 1) / C0, batch), C0 * FftShape<N>::N2, 0, s>>>(fa);
    return launch_status("k_psf_rows");
}

template <int N>
static int launch_psf_cols(const PsfFastArgs& fa, int batch, hipStream_t s) {
    constexpr int C0 = FftShape<N>::C0;
    const int C = C0 < fa.g.nx2 ? C0 : fa.g.nx2;
    const dim3 grid(fa.g.px / C, fa.g.py / N, batch);
    const unsigned threads = C * FftShape<N>::N2;
    k_psf_cols<N, false><<<grid, threads, 0, s>>>(fa, C);
    int st = launch_status("k_psf_cols(peak)");
    if (st) return st;
    k_psf_cols<N, true><<<grid, threads, 0, s>>>(fa, C);
    return launch_status("k_psf_cols");
}

// ---- line transforms (pad 8 / 16): whole output rows per store ----
//
// The same F[ko][lo] (up to its unit-modulus phases) in two passes of one kernel family:
//   pass 1, pupil columns: G[b][ko] = sum_a (-1)^a U0[a][b] W_py^(ko a)   (b < ex; G is ex x py,
//                          contiguous in ko)
//   pass 2, plane rows:    X[ko][lo] = sum_b (-1)^b G[b][ko] W_px^(lo b),   psf = |X dA|^2 / Imax
// Each line is a P = N PAD-point transform of N inputs, decimated in time so that every thread
// ends with whole output columns j (lanes consecutive in j, so each store instruction of pass 2
// writes 64 consecutive doubles of one psf row):
//   X[j + N r] = sum_{s<PAD} W_PAD^(s r) (W_P^(s j) Y_s[j])                       stage 2
//   Y_s[t + PAD u] = sum_{q<Q} (g[PAD q + s] W_N^(q t)) W_Q^(q u),  Q = N / PAD     stage 1
// Stage 1 runs SIG values of s at a time through LDS: Q <= SIG, whole Q-point DFTs per thread;
// Q = SIG Q2 (N >= 256 at pad 16), a SIG x Q2 four-step with one more exchange. Thread j gathers
// its Y_s[j], applies W_P^(s j) (powers of one table entry) and runs the PAD-point DFT in
// registers. Pass 2 runs twice: the peak, then the normalised write (its only HBM traffic is the
// output and one read of G). Workgroups are persistent over lines, prefetching the next line's
// inputs, and walk an XCD's share of the lines contiguously (pass 2's reads of G are 16-byte
// pieces of 128-byte lines shared by 8 neighbouring rows).
enum { kLinePupil = 0, kLinePeak = 1, kLineWrite = 2, kLineWriteE = 3, kLinePeak32 = 4 };
#ifndef AKB_PSF_NT
#define AKB_PSF_NT 1  // nontemporal psf stores (the stream must not evict G's lines): 0 for A/B
#endif
// The peak, fp32 route (AKB_PSF_PEAK=f32; the row-bound route below replaced it as the default on
// large planes): kLinePeak32 runs pass 2 in fp32 (half the LDS bytes, twice the VALU rate) for each
// row's max of |F|^2; the rows within kPeakSlack of the fp32 peak (the fp32 transform's error is
// ~1e-6 of the peak, its worst-case bound ~1e-3 at 1024-point lines) are re-run in fp64
// (kLinePeak over that list), which gives the exact max. Non-finite or zero peaks, or more than a
// quarter of the rows within the slack, take the fp64 pass over every row.
constexpr float kPeakSlack = 0.0625f;

template <typename R>
struct Cx;
template <>
struct Cx<double> {
    using T = double2;
    __device__ static double2 mk(double x, double y) { return make_double2(x, y); }
};
template <>
struct Cx<float> {
    using T = float2;
    __device__ static float2 mk(float x, float y) { return make_float2(x, y); }
};

template <typename R>
__device__ __forceinline__ typename Cx<R>::T cmul_r(typename Cx<R>::T a, typename Cx<R>::T b) {
    return Cx<R>::mk(fma(a.x, b.x, -(a.y * b.y)), fma(a.x, b.y, a.y * b.x));
}

// dft_reg_br with fused multiply-adds in precision R
template <int M, typename R>
__device__ __forceinline__ void dft_br(typename Cx<R>::T (&t)[M]) {
    using V = typename Cx<R>::T;
#pragma unroll
    for (int h = 1; h < M; h <<= 1) {
#pragma unroll
        for (int i = 0; i < M; i += 2 * h) {
#pragma unroll
            for (int k = 0; k < h; ++k) {
                const V x = t[i + k];
                V y = t[i + k + h];
                if (k != 0) {
                    if (2 * k == h) {
                        y = Cx<R>::mk(y.y, -y.x);
                    } else {
                        const int wi = k * (16 / h);
                        y = cmul_r<R>(y, Cx<R>::mk((R)kW32re[wi], (R)kW32im[wi]));
                    }
                }
                t[i + k] = Cx<R>::mk(x.x + y.x, x.y + y.y);
                t[i + k + h] = Cx<R>::mk(x.x - y.x, x.y - y.y);
            }
        }
    }
}

template <int N, int PAD>
struct LineShape {
    static constexpr int SIG = 8;
    static constexpr int CH = PAD / SIG;
    static constexpr int Q = N / PAD;
    static constexpr bool kFour = Q > SIG;
    static constexpr int Q2 = kFour ? Q / SIG : 1;
    static constexpr int LINES = N >= 256 ? 1 : 256 / N;
    static constexpr int kThreads = N * LINES;
    static constexpr int TS = SIG * PAD;  // stage-1 tasks (s, t) per chunk and line
    static constexpr int kTab = kFour ? Q2 * PAD + SIG * PAD + Q2 * SIG : Q * PAD;
    static_assert(Q >= 1 && Q2 <= SIG && PAD % SIG == 0, "line transform shape");
};

// threads of a workgroup: the 1024-point fp64 lines run two lanes j and j + 512 per thread in
// 512-thread workgroups (a 1024-thread workgroup caps a thread at 128 VGPRs, and a lane's sixteen
// outputs held across the second chunk's transform spilled past it; at 512 the cap is 256)
template <int N, int PAD, int MODE>
struct LineThreads {
    static constexpr int kLanes = (N >= 1024 && MODE != kLinePeak32) ? 2 : 1;
    static constexpr int kThreads = LineShape<N, PAD>::kThreads / kLanes;
    static_assert(kLanes == 1 || (LineShape<N, PAD>::LINES == 1 && kThreads % PAD == 0), "lane split");
};

struct PsfLineArgs {
    const double* opd;
    const double* amp;
    const double* wy;
    const double* wx;
    double wmax;
    double kphase[8];
    PsfGeom g;
    const double2* Wx;  // W_px table
    const double2* Wy;  // W_py table
    double2* G;         // (batch, ex, py)
    double dA;
    const double* pitch;
    double* psf;
    double2* efield;
    double* imax;        // Imax = max |F dA|^2 per batch entry (written by the write pass)
    double* umax;        // max |F|^2 per batch entry (workspace; pass 1 zeroes it)
    unsigned* umax32;    // fp32 peak pass: max |F|^2 (float bits) per batch entry
    float* rowmax32;     // fp32 peak pass: (batch, py) row maxima
    int* cand;           // (batch, py) rows for the fp64 peak pass
    int* cand_n;         // per batch entry: their count, or -1 for every row
    double* ubound;      // row-bound route: (batch, py) bounds B[ko] >= max_lo |F[ko][lo]|^2
    double* ubmax;       // row-bound route: per batch entry max B, NaN when the route is off
    double* bpart;       // select route: (batch, npart, py) sum over a pass-1 workgroup's columns of |G|
    double2* spart;      // select route: (batch, npart, 32) its columns' part of F at the kSel samples
    int npart;           // select route: pass 1's workgroup count
    int ngroups;         // line groups (LINES lines each) per batch entry
};

// The select route to the peak (the default below 2^24 points). Pass 1 also leaves, per workgroup,
// the sums over its pupil columns x of |G[x][ko]| for every row and of (-1)^x G[x][ko] W^(lo x) at
// a 5 x 5 grid of samples around the plane's centre (ko = py/2 - 2 .. py/2 + 2, lo likewise: the
// pupil's zero frequency, where a focused PSF peaks). The peak pass sums those parts in a fixed
// order in every workgroup: B[ko] = (sum_x |G[x][ko]|)^2 (1 + 2^-20) bounds every |F|^2 it computes
// in row ko (the row-bound argument below), and each sample S gives M_low = (|S| - d)^2 (1 - 2^-30)
// with d = 2^-30 sum_x |G[x][ko]|, below the |F|^2 the pass computes at that sample (both sums'
// roundings are ~1e-13 of sum_x |G|), so below the max. A row with B < M_low cannot hold the max:
// each workgroup transforms only its rows with B >= M_low (the peak row among them), all rows when
// M_low is not a positive finite number (dark, NaN or infinite field). The max is therefore the
// all-rows pass's exactly, with no launch beyond the three passes.
constexpr int kSel = 25;
constexpr int kSelRows = 256;
constexpr double kBoundMarginSel = 1.0 + 0x1p-20;

template <int N, int PAD, int MODE>
__global__ void __launch_bounds__((LineThreads<N, PAD, MODE>::kThreads)) k_psf_line(PsfLineArgs A) {
    AKB_CHAIN_PRIORITY();
    using S = LineShape<N, PAD>;
    constexpr int LPT = LineThreads<N, PAD, MODE>::kLanes, NT = LineThreads<N, PAD, MODE>::kThreads;
    using R = typename std::conditional<MODE == kLinePeak32, float, double>::type;
    using V = typename Cx<R>::T;
    constexpr int SIG = S::SIG, Q = S::Q, Q2 = S::Q2, LINES = S::LINES, TS = S::TS;
    constexpr int LQ = ilog2_c(Q), LS = ilog2_c(SIG), LQ2 = ilog2_c(Q2);
    __shared__ V Yc[LINES * SIG * N];
    __shared__ V gl[LINES * N];
    __shared__ V tab[S::kTab];
    __shared__ double wm[NT / 64];
    // select route (pass 1 of planes up to 4096 rows: per-workgroup row sums; the peak pass: its rows)
    constexpr int BS = (MODE == kLinePupil && N * PAD <= 4096) ? N * PAD : 1;
    constexpr bool kSelPeak = MODE == kLinePeak;
    __shared__ double Bsum[BS];
    __shared__ double2 Gs[MODE == kLinePupil ? LINES : 1][5];
    __shared__ int Lc[MODE == kLinePupil ? LINES : 1];
    __shared__ int lrows[kSelPeak ? kSelRows : 1];
    __shared__ double ssum[kSelPeak ? 3 * kSel + kSelRows : 1];  // samples (re, im, sum |G|), row bounds
    __shared__ int lcount;
    __shared__ double msel;
    const PsfGeom g = A.g;
    const int b = blockIdx.y;
    const bool sel1 = BS > 1 && A.bpart != nullptr;  // pass 1 leaves the select route's parts
    const double2* WP = MODE == kLinePupil ? A.Wy : A.Wx;
    const int line = threadIdx.x / N, i0 = threadIdx.x % N;
    int i = i0, q2 = i0 / TS;  // the current lane (below: lane(h)) and its four-step row
    int t = i0 % PAD;          // the same for every lane of a thread (NT is a multiple of PAD)
    // lines of this pass: pupil columns (pass 1), psf rows, or the fp64 peak pass's row list
    int nl = MODE == kLinePupil ? g.nx2 : g.py;
    const int* rows = nullptr;
    if (MODE == kLinePeak && A.cand) {
        const int cn = A.cand_n[b];
        if (cn >= 0) {
            nl = cn;
            rows = A.cand + (int64_t)b * g.py;
        }
    }
    if (MODE == kLinePupil && blockIdx.x == 0 && threadIdx.x == 0) {
        A.umax[b] = 0.0;  // pass 2 follows
        A.umax32[b] = 0u;
    }
    // this workgroup's line groups: an XCD's contiguous share, slot-strided within it
    int ngr = rows ? (nl + LINES - 1) / LINES : A.ngroups;
    const int nwg = gridDim.x;
    int base = 0, slot = blockIdx.x, nslot = nwg, RR = ngr;
    if ((nwg & 7) == 0) {
        RR = (ngr + 7) / 8;
        base = (blockIdx.x & 7) * RR;
        slot = blockIdx.x >> 3;
        nslot = nwg >> 3;
    }
    auto group_at = [&](int k) {
        const int o = slot + k * nslot;
        const int gi = base + o;
        return (o < RR && gi < (rows ? (nl + LINES - 1) / LINES : ngr)) ? gi : -1;
    };
    double2 sacc = make_double2(0.0, 0.0);
    if (sel1) {
        for (int k = threadIdx.x; k < BS; k += NT) Bsum[k] = 0.0;
        if (group_at(0) < 0) {  // no columns here: its parts are zero
            double* bp = A.bpart + ((int64_t)b * A.npart + blockIdx.x) * g.py;
            for (int k = threadIdx.x; k < g.py; k += NT) bp[k] = 0.0;
            if (threadIdx.x < kSel) A.spart[((int64_t)b * A.npart + blockIdx.x) * 32 + threadIdx.x] = sacc;
            return;
        }
    }
    if (kSelPeak && A.bpart && !rows) {
        // M_low from the samples and the bounds of this workgroup's rows: the workgroups' parts
        // summed by all threads at once (LDS atomics: any order gives a valid bound, the margins
        // cover the rounding; a long per-thread chain of L2 loads would be the kernel's critical path)
        const int np = A.npart;
        const int64_t pb = (int64_t)b * np;
        int nmine = 0;
        for (int k = 0; group_at(k) >= 0; ++k) nmine += LINES;
        const bool fits = nmine <= kSelRows;
        for (int e = threadIdx.x; e < 3 * kSel + kSelRows; e += NT) ssum[e] = 0.0;
        if (threadIdx.x == 0) lcount = 0;
        __syncthreads();
        for (int e = threadIdx.x; e < kSel * np; e += NT) {
            const int k = e % kSel, w = e / kSel;
            const double2 tv = A.spart[(pb + w) * 32 + k];
            atomicAdd(&ssum[k], tv.x);
            atomicAdd(&ssum[kSel + k], tv.y);
            atomicAdd(&ssum[2 * kSel + k], A.bpart[(pb + w) * g.py + g.py / 2 - 2 + k / 5]);
        }
        if (fits)
            for (int e = threadIdx.x; e < nmine * np; e += NT) {
                const int q = e / np, w = e - (e / np) * np;
                const int row = group_at(q / LINES) * LINES + q % LINES;
                if (row < nl) atomicAdd(&ssum[3 * kSel + q], A.bpart[(pb + w) * g.py + row]);
            }
        __syncthreads();
        double mk = 0.0;
        if (threadIdx.x < kSel) {
            const double sx = ssum[threadIdx.x], sy = ssum[kSel + threadIdx.x], bs = ssum[2 * kSel + threadIdx.x];
            const double as = sqrt(fma(sx, sx, sy * sy)), dl = bs * 0x1p-30;
            mk = as > dl ? ((as - dl) * (as - dl)) * (1.0 - 0x1p-30) : (as == as && dl == dl ? 0.0 : as + dl);
        }
        if (threadIdx.x < 64) {
            for (int off = 32; off > 0; off >>= 1) mk = dmax_nan(mk, __shfl_down(mk, off));
            if (threadIdx.x == 0) msel = mk;
        }
        __syncthreads();
        const double M = msel;
        const bool all = !(M > 0.0) || !isfinite(M);
        // this workgroup's rows (the all-rows pass's assignment): keep those with B >= M_low
        if (!all && fits) {
            for (int q = threadIdx.x; q < nmine; q += NT) {
                const int row = group_at(q / LINES) * LINES + q % LINES;
                const double bs = ssum[3 * kSel + q];
                if (row < nl && !((bs * bs) * kBoundMarginSel < M)) lrows[atomicAdd(&lcount, 1)] = row;
            }
            __syncthreads();
            nl = lcount;
            rows = lrows;
            base = 0;
            slot = 0;
            nslot = 1;
            RR = (nl + LINES - 1) / LINES;
        }
    }
    // a workgroup without lines (the peak rounds' short row lists) leaves before its tables
    if (group_at(0) < 0) return;
    // stage-1 twiddles, W_N^m = W_P^(PAD m): four-step, TA[q2][t] = W_N^(q2 t),
    // TB[q1][t] = W_N^(q1 Q2 t), TQ[q2][k1] = W_Q^(q2 k1); one-step, T2[q][t] = W_N^(q t)
    V* TA = tab;
    V* TB = tab + Q2 * PAD;
    V* TQ = tab + Q2 * PAD + SIG * PAD;
    for (int e = threadIdx.x; e < S::kTab; e += NT) {
        int m;
        if (S::kFour) {
            if (e < Q2 * PAD)
                m = (e / PAD) * (e % PAD);
            else if (e < Q2 * PAD + SIG * PAD)
                m = ((e - Q2 * PAD) / PAD) * Q2 * ((e - Q2 * PAD) % PAD);
            else
                m = PAD * ((e - Q2 * PAD - SIG * PAD) / SIG) * ((e - Q2 * PAD - SIG * PAD) % SIG);
        } else {
            m = (e / PAD) * (e % PAD);
        }
        const double2 w = WP[(int64_t)PAD * m];
        tab[e] = Cx<R>::mk((R)w.x, (R)w.y);
    }
    const double dA = A.pitch ? A.pitch[0] * A.pitch[1] : A.dA;
    // psf = |F dA|^2 / Imax = |F|^2 / max |F|^2 (unnormalised |F dA|^2 when Imax is not > 0, as
    // psf_fft.py:120-122); Imax itself goes to the caller's imax
    double scale = 1.0, sq = 1.0;
    if (MODE == kLineWrite || MODE == kLineWriteE) {
        const double um = A.umax[b];
        const double imx = um * dA * dA;
        scale = imx > 0.0 ? 1.0 / um : dA * dA;
        sq = sqrt(imx > 0.0 ? imx : 1.0);
        if (blockIdx.x == 0 && threadIdx.x == 0) A.imax[b] = imx;
    }
    const double sgn = ((g.ny2 / 2 + g.nx2 / 2) & 1) ? -1.0 : 1.0;

    auto line_of = [&](int grp) {  // -1: none
        const int idx = grp * LINES + line;
        if (grp < 0 || idx >= nl) return -1;
        return rows ? rows[idx] : idx;
    };
    // inputs: pass 1, (opd, amp) of pupil element (a = i, column = line); pass 2, G[x = i][ko = line]
    auto fetch = [&](int L) {
        double2 r = make_double2(0.0, 0.0);
        if (L < 0) return r;
        if (MODE == kLinePupil) {
            if (i < g.ny && L < g.nx) {
                const int64_t pi = (int64_t)i * g.nx + L;
                r.x = A.opd[pi];
                r.y = A.amp ? A.amp[pi] : (isfinite(r.x) ? 1.0 : 0.0);
            }
        } else {
            r = A.G[((int64_t)b * g.nx2 + i) * g.py + L];
        }
        return r;
    };
    auto input = [&](double2 r, int L) {
        double re = r.x, im = r.y;
        if (MODE == kLinePupil) {
            re = 0.0;
            im = 0.0;
            if (L >= 0 && i < g.ny && L < g.nx) {
                double o = r.x, amp = r.y;
                if (!isfinite(amp)) amp = 0.0;
                if (!isfinite(o)) o = 0.0;
                double sn, cs;
                sincos(A.kphase[b] * o, &sn, &cs);
                re = amp * cs - 0.0 * sn;
                im = amp * sn + 0.0 * cs;
                if (A.wy) {
                    const double w = (A.wy[i] * A.wx[L]) / A.wmax;
                    const double x0 = re, y0 = im;
                    re = x0 * w - y0 * 0.0;
                    im = x0 * 0.0 + y0 * w;
                }
            }
        }
        if (i & 1) {
            re = -re;
            im = -im;
        }
        return Cx<R>::mk((R)re, (R)im);
    };

    double m = 0.0, nan_sum = 0.0;
    unsigned m32 = 0u;
    auto lane = [&](int h) {  // lane h of this thread: j = i0 + h NT
        int x = i0;
        // two lanes: the lane index opaque at each phase, so the LDS addresses derived from it are
        // formed where they are used instead of hoisted out of the line loop (four phases x eight
        // addresses x two lanes held across every line would fill the registers)
        if constexpr (LPT > 1) asm volatile("" : "+v"(x));
        i = x + h * NT;
        q2 = i / TS;
        t = i % PAD;
    };
    int grp = group_at(0);
    double2 pre[LPT];
#pragma unroll
    for (int h = 0; h < LPT; ++h) {
        lane(h);
        pre[h] = fetch(line_of(grp));
    }
    for (int k = 0; grp >= 0; ++k) {
        const int L = line_of(grp);
        const int next = group_at(k + 1);
        __syncthreads();  // the previous group is done with gl / Yc / wm (and the tables are in)
#pragma unroll
        for (int h = 0; h < LPT; ++h) {
            lane(h);
            gl[line * N + i] = input(pre[h], L);
            pre[h] = fetch(line_of(next));
        }
        __syncthreads();
        V v[LPT][PAD];
        // a lane's outputs, formed as soon as its last chunk is done (its registers then free for
        // the next lane)
        auto emit = [&](const V (&vh)[PAD]) {
            if constexpr (MODE == kLinePupil) {
                if (L >= 0) {
                    double2* Gl = A.G + ((int64_t)b * g.nx2 + L) * g.py + i;
#pragma unroll
                    for (int r = 0; r < PAD; ++r) Gl[(int64_t)N * r] = vh[r];
                }
                if constexpr (BS > 1) {
                    if (sel1) {
                        // |G| into the row sums, one line after the other (a fixed order); the sample
                        // rows' values to LDS
                        for (int ln = 0; ln < LINES; ++ln) {
                            __syncthreads();
                            if (line == ln && L >= 0) {
#pragma unroll
                                for (int r = 0; r < PAD; ++r) Bsum[i + N * r] += sqrt(fma(vh[r].x, vh[r].x, vh[r].y * vh[r].y));
                            }
                        }
                        if (i == 0) Lc[line] = L;
#pragma unroll
                        for (int r = 0; r < PAD; ++r) {
                            const int d = i + N * r - (N * PAD / 2 - 2);
                            if (d >= 0 && d < 5) Gs[line][d] = L >= 0 ? vh[r] : make_double2(0.0, 0.0);
                        }
                        __syncthreads();
                        if (threadIdx.x < kSel) {  // sample (ko = py/2 - 2 + k / 5, lo = px/2 - 2 + k % 5)
                            const int dk = threadIdx.x / 5, lo = g.px / 2 - 2 + threadIdx.x % 5;
                            for (int ln = 0; ln < LINES; ++ln) {
                                const int x = Lc[ln];
                                if (x < 0) continue;
                                double2 t = cmul(Gs[ln][dk], A.Wx[((int64_t)lo * x) % g.px]);
                                if (x & 1) t = make_double2(-t.x, -t.y);
                                sacc.x += t.x;
                                sacc.y += t.y;
                            }
                        }
                    }
                }
            } else if constexpr (MODE == kLinePeak32) {
                // this row's max (uint order of non-negative floats is numeric, NaN above +inf)
                unsigned mr = 0u;
#pragma unroll
                for (int r = 0; r < PAD; ++r) {
                    const float U = fmaf(vh[r].x, vh[r].x, vh[r].y * vh[r].y);
                    mr = max(mr, __float_as_uint(U));
                }
                constexpr int W = N < 64 ? N : 64;
#pragma unroll
                for (int off = 1; off < W; off <<= 1) mr = max(mr, (unsigned)__shfl_xor((int)mr, off));
                if (N > 64) {
                    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = (double)__uint_as_float(mr);
                    __syncthreads();
                    if (i == 0)
                        for (int w = 1; w < N / 64; ++w) mr = max(mr, __float_as_uint((float)wm[(threadIdx.x >> 6) + w]));
                }
                if (i == 0 && L >= 0) {
                    A.rowmax32[(int64_t)b * g.py + L] = __uint_as_float(mr);
                    m32 = max(m32, mr);
                }
            } else {
              if (L >= 0) {
                double* Pr = A.psf + ((int64_t)b * g.py + L) * g.px + i;
                double2* Er = A.efield + ((int64_t)b * g.py + L) * g.px + i;
#pragma unroll
                for (int r = 0; r < PAD; ++r) {
                    const double U = fma(vh[r].x, vh[r].x, vh[r].y * vh[r].y);
                    if (MODE == kLinePeak) {
                        m = fmax(m, U);
                        nan_sum += U;  // NaN iff some U is NaN (U >= 0): numpy's max propagates it
                    } else {
                        if (AKB_PSF_NT)
                            __builtin_nontemporal_store(U * scale, Pr + N * r);
                        else
                            Pr[N * r] = U * scale;
                        if (MODE == kLineWriteE) {
                            const double re = vh[r].x * dA, im = vh[r].y * dA;
                            const int lo = i + N * r;
                            const double2 py_ph = A.Wy[((int64_t)L * (g.ny2 / 2)) % g.py];
                            const double2 px_ph = A.Wx[((int64_t)lo * (g.nx2 / 2)) % g.px];
                            double2 e = cmul(make_double2(re, im), make_double2(py_ph.x, -py_ph.y));
                            e = cmul(e, make_double2(px_ph.x, -px_ph.y));
                            Er[N * r] = make_double2(sgn * e.x / sq, sgn * e.y / sq);
                        }
                    }
                }
              }
            }
        };
        V w1[LPT], wch[LPT];
#pragma unroll
        for (int h = 0; h < LPT; ++h) {
            const double2 w1d = WP[i0 + h * NT];  // W_P^j (reloaded per line: fewer registers held across it)
            w1[h] = Cx<R>::mk((R)w1d.x, (R)w1d.y);
            wch[h] = S::CH == 1 ? w1[h] : cmul_r<R>(w1[h], w1[h]);
        }
        V* Yl = Yc + line * SIG * N;
        const V* gll = gl + line * N;
#pragma unroll
        for (int c = 0; c < S::CH; ++c) {
            if constexpr (!S::kFour) {
#pragma unroll
                for (int h = 0; h < LPT; ++h) {
                    lane(h);
#pragma unroll
                    for (int kk = 0; kk < SIG / Q; ++kk) {
                        const int s_l = (i + kk * N) / PAD, s = S::CH * s_l + c;
                        V w[Q];
#pragma unroll
                        for (int q = 0; q < Q; ++q) {
                            const V x = gll[PAD * q + s];
                            w[bitrev_c(q, LQ)] = q ? cmul_r<R>(x, tab[q * PAD + t]) : x;
                        }
                        dft_br<Q, R>(w);
#pragma unroll
                        for (int u = 0; u < Q; ++u) Yl[s_l * N + t + PAD * u] = w[u];
                    }
                }
            } else {
#pragma unroll
                for (int h = 0; h < LPT; ++h) {
                    lane(h);
                    const int task = i % TS;
                    const int s_l = task / PAD, s = S::CH * s_l + c;
                    V w[SIG];
#pragma unroll
                    for (int q1 = 0; q1 < SIG; ++q1) {
                        const V x = gll[PAD * (q1 * Q2 + q2) + s];
                        w[bitrev_c(q1, LS)] = q1 ? cmul_r<R>(x, TB[q1 * PAD + t]) : x;
                    }
                    dft_br<SIG, R>(w);
                    const V tw0 = TA[q2 * PAD + t];  // W_N^(q2 t) W_Q^(q2 k1)
#pragma unroll
                    for (int k1 = 0; k1 < SIG; ++k1) {
                        const V tw = k1 ? cmul_r<R>(tw0, TQ[q2 * SIG + k1]) : tw0;
                        Yl[(k1 * Q2 + q2) * TS + task] = cmul_r<R>(w[k1], tw);
                    }
                    if (h + 1 < LPT) __builtin_amdgcn_sched_barrier(0);
                }
                __syncthreads();
                {
                    V w[LPT][SIG / Q2][Q2];
#pragma unroll
                    for (int h = 0; h < LPT; ++h) {
                        lane(h);
                        const int task = i % TS, kg = i / TS;
#pragma unroll
                        for (int e = 0; e < SIG / Q2; ++e) {
                            const int k1 = kg + Q2 * e;
#pragma unroll
                            for (int ii = 0; ii < Q2; ++ii)
                                w[h][e][ii] = Yl[(k1 * Q2 + bitrev_c(ii, LQ2)) * TS + task];
                        }
                    }
                    __syncthreads();
#pragma unroll
                    for (int h = 0; h < LPT; ++h) {
                        lane(h);
                        const int task = i % TS, kg = i / TS;
                        const int s_l = task / PAD;
#pragma unroll
                        for (int e = 0; e < SIG / Q2; ++e) {
                            dft_br<Q2, R>(w[h][e]);
                            const int k1 = kg + Q2 * e;
#pragma unroll
                            for (int k2 = 0; k2 < Q2; ++k2) Yl[s_l * N + t + PAD * (k1 + SIG * k2)] = w[h][e][k2];
                        }
                        if (h + 1 < LPT) __builtin_amdgcn_sched_barrier(0);
                    }
                }
            }
            __syncthreads();
            // stage 2 of this chunk's s = CH s' + c: W_P^(s j) as powers of W_P^(CH j) (at most
            // SIG - 1 roundings), the SIG-point DFT over s'
#pragma unroll
            for (int h = 0; h < LPT; ++h) {
                lane(h);
                V a[SIG];
                {
                    V p = c ? w1[h] : Cx<R>::mk((R)1, (R)0);
#pragma unroll
                    for (int s_l = 0; s_l < SIG; ++s_l) {
                        const V y = Yl[s_l * N + i];
                        a[bitrev_c(s_l, LS)] = (c == 0 && s_l == 0) ? y : cmul_r<R>(y, p);
                        if (s_l + 1 < SIG) p = (c == 0 && s_l == 0) ? wch[h] : cmul_r<R>(p, wch[h]);
                    }
                }
                dft_br<SIG, R>(a);
                if constexpr (S::CH == 1) {
#pragma unroll
                    for (int r = 0; r < SIG; ++r) v[h][r] = a[r];
                } else {
                    // PAD = 2 SIG: X[r] = A0[r] + W_PAD^r A1[r], X[r + SIG] = A0[r] - W_PAD^r A1[r]
                    if (c == 0) {
#pragma unroll
                        for (int r = 0; r < SIG; ++r) v[h][r] = a[r];
                    } else {
#pragma unroll
                        for (int r = 0; r < SIG; ++r) {
                            const int wi = r * (32 / PAD);
                            const V tt = r ? cmul_r<R>(a[r], Cx<R>::mk((R)kW32re[wi], (R)kW32im[wi])) : a[r];
                            const V x0 = v[h][r];
                            v[h][r] = Cx<R>::mk(x0.x + tt.x, x0.y + tt.y);
                            v[h][r + SIG] = Cx<R>::mk(x0.x - tt.x, x0.y - tt.y);
                        }
                    }
                }
                if (c + 1 == S::CH) emit(v[h]);
                if (h + 1 < LPT) __builtin_amdgcn_sched_barrier(0);  // one lane after the other
            }
            if (c + 1 < S::CH) __syncthreads();
        }
        grp = next;
    }
    if constexpr (BS > 1) {
        if (sel1) {
            __syncthreads();
            double* bp = A.bpart + ((int64_t)b * A.npart + blockIdx.x) * g.py;
            for (int k = threadIdx.x; k < g.py; k += NT) bp[k] = Bsum[k];
            if (threadIdx.x < kSel) A.spart[((int64_t)b * A.npart + blockIdx.x) * 32 + threadIdx.x] = sacc;
        }
    }
    if (MODE == kLinePeak) {
        if (nan_sum != nan_sum) m = nan_sum;
        for (int off = 32; off > 0; off >>= 1) m = dmax_nan(m, __shfl_down(m, off));
        __syncthreads();
        if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int w = 1; w < NT / 64; ++w) m = dmax_nan(m, wm[w]);
            atomic_max_nonneg(A.umax + b, m);
        }
    } else if (MODE == kLinePeak32) {
        // thousands of workgroups meet on one word: only a new maximum issues the atomic
        if (m32 > __hip_atomic_load(A.umax32 + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(A.umax32 + b, m32);
    }
}

// the fp64 peak pass's rows: those whose fp32 max is within kPeakSlack of the fp32 peak (one
// workgroup per batch entry; -1 = every row)
__global__ void __launch_bounds__(1024) k_psf_peak_rows(PsfLineArgs A, int limit) {
    __shared__ int cnt;
    const int b = blockIdx.x, py = A.g.py;
    const float M = __uint_as_float(A.umax32[b]);
    const bool all = !(M > 0.0f) || !isfinite(M);
    const float thr = M * (1.0f - kPeakSlack);
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    if (!all) {
        const float* rm = A.rowmax32 + (int64_t)b * py;
        int* cd = A.cand + (int64_t)b * py;
        for (int r = threadIdx.x; r < py; r += blockDim.x) {
            if (rm[r] >= thr) {
                const int k = atomicAdd(&cnt, 1);
                if (k < limit) cd[k] = r;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) A.cand_n[b] = (all || cnt > limit) ? -1 : cnt;
}

// The row-bound route to the peak (the default). Pass 2 computes row ko of F as
// X[lo] = sum_x (-1)^x G[x][ko] W^(lo x), so |X[lo]| <= sum_x |G[x][ko]| for every lo: B[ko], that
// sum squared times 1 + 2^-20, bounds every |F|^2 the kernel computes for the row (the rounding of
// a line transform and of the sum are ~1e-13 of it), and no row whose bound lies below some
// computed |F|^2 holds the peak. Round 1 runs the fp64 peak pass over the rows with B >= B_max / 2
// (a focused PSF's peak row is among them: its coherent sum reaches B); round 2 over the rest with
// B >= round 1's max M1. Every row that could hold the peak is in one of the rounds, each row's
// values are the write pass's bits, so the max is the all-rows pass's max exactly. A non-finite or
// zero B_max (NaN or infinite field, dark pupil) turns the route off: round 1 takes every row.
// Measured on the example's 1024^2 pupil: 1 of 16384 rows; ~2.5 % with 3 waves of aberration.
constexpr double kBoundMargin = 1.0 + 0x1p-20;
constexpr double kBoundTheta = 0.5;

// B per row: one workgroup per 64 rows and batch entry, sixteen waves over the pupil columns,
// summed in a fixed order
__global__ void __launch_bounds__(1024) k_psf_rowbound(PsfLineArgs A) {
    __shared__ double red[16][64];
    const PsfGeom g = A.g;
    const int b = blockIdx.y;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ko = blockIdx.x * 64 + lane;
    double s = 0.0;
    if (ko < g.py) {
        const double2* Gp = A.G + (int64_t)b * g.nx2 * g.py + ko;
#pragma unroll 4
        for (int x = w; x < g.nx2; x += 16) {
            const double2 v = Gp[(int64_t)x * g.py];
            s += sqrt(fma(v.x, v.x, v.y * v.y));
        }
    }
    red[w][lane] = s;
    __syncthreads();
    if (w == 0 && ko < g.py) {
        double t = red[0][lane];
        for (int k = 1; k < 16; ++k) t += red[k][lane];
        A.ubound[(int64_t)b * g.py + ko] = (t * t) * kBoundMargin;
    }
}

// B_max and round 1's rows (one workgroup per batch entry)
__global__ void __launch_bounds__(1024) k_psf_bound_rows1(PsfLineArgs A) {
    __shared__ double wmx[16];
    __shared__ int cnt;
    const int b = blockIdx.x, py = A.g.py;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const double* ub = A.ubound + (int64_t)b * py;
    double m = 0.0;
    for (int r = threadIdx.x; r < py; r += blockDim.x) m = dmax_nan(m, ub[r]);
    for (int off = 32; off > 0; off >>= 1) m = dmax_nan(m, __shfl_down(m, off));
    if (lane == 0) wmx[w] = m;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    m = wmx[0];
    for (int k = 1; k < 16; ++k) m = dmax_nan(m, wmx[k]);
    const bool on = isfinite(m) && m > 0.0;
    if (on) {
        const double thr = m * kBoundTheta;
        int* cd = A.cand + (int64_t)b * py;
        for (int r = threadIdx.x; r < py; r += blockDim.x)
            if (ub[r] >= thr) cd[atomicAdd(&cnt, 1)] = r;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        A.ubmax[b] = on ? m : __builtin_nan("");
        A.cand_n[b] = on ? cnt : -1;
    }
}

// round 2's rows: B below round 1's threshold but not below its max M1 (none when the route is
// off; a NaN M1 is already the answer)
__global__ void __launch_bounds__(1024) k_psf_bound_rows2(PsfLineArgs A) {
    __shared__ int cnt;
    const int b = blockIdx.x, py = A.g.py;
    const double M = A.ubmax[b], m1 = A.umax[b];
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    if (M == M) {
        const double thr = M * kBoundTheta;
        const double* ub = A.ubound + (int64_t)b * py;
        int* cd = A.cand + (int64_t)b * py;
        for (int r = threadIdx.x; r < py; r += blockDim.x) {
            const double u = ub[r];
            if (u < thr && u >= m1) cd[atomicAdd(&cnt, 1)] = r;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) A.cand_n[b] = cnt;
}

#ifndef AKB_PSF_SEL_WGS
#define AKB_PSF_SEL_WGS 128
#endif
constexpr int kSelPeakWgs = AKB_PSF_SEL_WGS;  // the select route's peak-pass grid (0: line_wgs)

// persistent workgroups per pass: the resident count (LDS / threads) x 256 CUs, a multiple of 8
template <int N, int PAD, typename R, int NT = LineShape<N, PAD>::kThreads>
static int line_wgs(int ngroups) {
    using S = LineShape<N, PAD>;
    const int lds = (int)(2 * sizeof(R)) * (S::LINES * S::SIG * N + S::LINES * N + S::kTab);
    int per_cu = (160 * 1024) / lds;
    const int by_threads = 2048 / NT;
    if (per_cu > by_threads) per_cu = by_threads;
    if (per_cu < 1) per_cu = 1;
    int w = 256 * per_cu;
    if (ngroups < w) w = ngroups >= 8 ? ngroups / 8 * 8 : ngroups;
    return w;
}

template <int N, int PAD, int MODE>
static int launch_psf_line(PsfLineArgs fa, int nlines, int batch, hipStream_t s) {
    using S = LineShape<N, PAD>;
    using R = typename std::conditional<MODE == kLinePeak32, float, double>::type;
    fa.ngroups = (nlines + S::LINES - 1) / S::LINES;
    using T = LineThreads<N, PAD, MODE>;
    int wgs = line_wgs<N, PAD, R, T::kThreads>(fa.ngroups);
    // the select route's peak pass: most of its workgroups only sum the bounds of their few rows
    // and leave (a focused PSF's peak rows are a handful), yet each needs a CU slot with its LDS
    // while the trace passes hold the CUs; a small grid (a multiple of 8: the XCD shares) takes
    // the slots the chain's reserved CUs have in one round
    if (MODE == kLinePeak && fa.bpart && !fa.cand && kSelPeakWgs > 0 && wgs > kSelPeakWgs) wgs = kSelPeakWgs;
    k_psf_line<N, PAD, MODE><<<dim3(wgs, batch), T::kThreads, 0, s>>>(fa);
    return launch_status(MODE == kLinePupil  ? "k_psf_line(pupil)"
                         : MODE == kLinePeak32 ? "k_psf_line(peak32)"
                         : MODE == kLinePeak   ? "k_psf_line(peak)"
                                               : "k_psf_line(write)");
}

// pass 1's workgroup count for a pupil of n-point columns at this pad (the select route's parts)
template <int N, int PAD>
static int pupil_pass_wgs(int nlines) {
    using S = LineShape<N, PAD>;
    return line_wgs<N, PAD, double, LineThreads<N, PAD, kLinePupil>::kThreads>((nlines + S::LINES - 1) / S::LINES);
}

// pad 16: lines of 16..1024; pad 8: 8..512 (Q = N / PAD <= 64)
#define AKB_LINE_SHAPES(X) \
    X(16, 16) X(32, 16) X(64, 16) X(128, 16) X(256, 16) X(512, 16) X(1024, 16) \
    X(8, 8) X(16, 8) X(32, 8) X(64, 8) X(128, 8) X(256, 8) X(512, 8)

static bool psf_line_ok(const PsfGeom& g, int pad) {
    if (getenv("AKB_PSF_ROCFFT")) return false;
    if (const char* e = getenv("AKB_PSF_PATH"))
        if (strcmp(e, "cols") == 0) return false;
    auto ok = [&](int n) {
#define AKB_CASE(NN, PP) if (n == NN && pad == PP) return true;
        AKB_LINE_SHAPES(AKB_CASE)
#undef AKB_CASE
        return false;
    };
    return ok(g.ny2) && ok(g.nx2) && (int64_t)g.py * g.px < (1LL << 31);
}

template <int MODE>
static int psf_line_dispatch(int n, int pad, const PsfLineArgs& fa, int nlines, int batch, hipStream_t s) {
#define AKB_CASE(NN, PP) \
    if (n == NN && pad == PP) return launch_psf_line<NN, PP, MODE>(fa, nlines, batch, s);
    AKB_LINE_SHAPES(AKB_CASE)
#undef AKB_CASE
    set_error("line PSF: unsupported line %d at pad %d", n, pad);
    return AKB_E_INVALID;
}

static int psf_line_pupil_wgs(int n, int pad, int nlines) {
#define AKB_CASE(NN, PP) \
    if (n == NN && pad == PP) return pupil_pass_wgs<NN, PP>(nlines);
    AKB_LINE_SHAPES(AKB_CASE)
#undef AKB_CASE
    return -1;
}

#define AKB_PSF_SIZES(X) X(8) X(16) X(32) X(64) X(128) X(256) X(512) X(1024)

static int psf_rows_dispatch(int n, const PsfFastArgs& fa, int batch, hipStream_t s) {
    switch (n) {
#define AKB_CASE(N) \
    case N:         \
        return launch_psf_rows<N>(fa, batch, s);
        AKB_PSF_SIZES(AKB_CASE)
#undef AKB_CASE
    }
    set_error("pruned PSF: unsupported row length %d", n);
    return AKB_E_INVALID;
}

static int psf_cols_dispatch(int n, const PsfFastArgs& fa, int batch, hipStream_t s) {
    switch (n) {
#define AKB_CASE(N) \
    case N:         \
        return launch_psf_cols<N>(fa, batch, s);
        AKB_PSF_SIZES(AKB_CASE)
#undef AKB_CASE
    }
    set_error("pruned PSF: unsupported column length %d", n);
    return AKB_E_INVALID;
}

static int ilog2_exact(int v) {
    if (v <= 0 || (v & (v - 1))) return -1;
    int l = 0;
    while ((1 << l) < v) ++l;
    return l;
}

static bool psf_fast_ok(const PsfGeom& g) {
    if (getenv("AKB_PSF_ROCFFT")) return false;
    const int ly = ilog2_exact(g.ny2), lx = ilog2_exact(g.nx2);
    // up to 256 at any pad; 512 / 1024 only at pad >= 8, where the padded plane rocFFT would
    // transform is 64x the pupil or more (their 32-point register DFTs run at one wave per SIMD
    // and lose to rocFFT on a small plane: 1024^2 pupil, pad 2: 193 vs 151 us)
    const int pad = g.px / g.nx2;
    const int lmax = pad >= 8 ? 10 : 8;
    return ly >= 3 && ly <= lmax && lx >= 3 && lx <= lmax && (int64_t)g.py * g.px < (1LL << 31);
}

static int64_t psf_fast_bytes(const PsfGeom& g, int batch) {
    return ((int64_t)batch * g.ny2 * g.px * 16 + 255) / 256 * 256;
}

// one 4-byte value per psf row and batch entry (fp32 row maxima, then the fp64 peak pass's rows)
static int64_t psf_line_rows_bytes(const PsfGeom& g, int batch) {
    return ((int64_t)batch * g.py * 4 + 255) / 256 * 256;
}

// the select route's per-workgroup parts (pass 1 has at most one workgroup per pupil column)
static bool psf_sel_ok(const PsfGeom& g) { return g.py <= 4096 && g.px <= 4096; }
static int64_t psf_sel_bytes(const PsfGeom& g, int batch) {
    if (!psf_sel_ok(g)) return 0;
    return (((int64_t)batch * g.nx2 * g.py * 8 + 255) / 256 * 256) + (int64_t)batch * g.nx2 * 32 * 16;
}

// W_P tables, built once per (device, P) and kept by the library (freed by akb_psf_release_plans)
static std::mutex g_tw_mu;
static std::map<std::pair<int, int>, double2*> g_tw;

static int get_twiddles(int P, hipStream_t s, const double2** out) {
    int dev = 0;
    AKB_HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_tw_mu);
    auto key = std::make_pair(dev, P);
    auto it = g_tw.find(key);
    if (it != g_tw.end()) {
        *out = it->second;
        return AKB_OK;
    }
    double2* W = nullptr;
    AKB_HIP_CHECK(hipMalloc(&W, (size_t)P * sizeof(double2)));
    k_psf_twiddle<<<(P + kBlock - 1) / kBlock, kBlock, 0, s>>>(W, P);
    int st = launch_status("k_psf_twiddle");
    if (st) return st;
    AKB_HIP_CHECK(hipStreamSynchronize(s));  // other streams may use the table right away
    g_tw[key] = W;
    *out = W;
    return AKB_OK;
}

// ---- rocFFT plan cache (thread-safe; the reference's _multi pattern runs one thread per GPU) ----

struct PlanEntry {
    rocfft_plan plan = nullptr;
    size_t work = 0;
};

static std::mutex g_plan_mu;
static std::map<std::tuple<int, int, int, int>, PlanEntry> g_plans;  // (device, py, px, batch)
static bool g_rocfft_ready = false;

static int get_plan(int py, int px, int batch, PlanEntry* out) {
    int dev = 0;
    AKB_HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_plan_mu);
    if (!g_rocfft_ready) {
        if (rocfft_setup() != rocfft_status_success) {
            set_error("rocfft_setup failed");
            return AKB_E_FFT;
        }
        g_rocfft_ready = true;
    }
    auto key = std::make_tuple(dev, py, px, batch);
    auto it = g_plans.find(key);
    if (it != g_plans.end()) {
        *out = it->second;
        return AKB_OK;
    }
    PlanEntry e;
    const size_t lengths[2] = {(size_t)px, (size_t)py};  // fastest dimension first
    rocfft_status st = rocfft_plan_create(&e.plan, rocfft_placement_inplace,
                                          rocfft_transform_type_complex_forward,
                                          rocfft_precision_double, 2, lengths, (size_t)batch, nullptr);
    if (st != rocfft_status_success) {
        set_error("rocfft_plan_create(%d x %d, batch %d) failed: %d", py, px, batch, (int)st);
        return AKB_E_FFT;
    }
    if (rocfft_plan_get_work_buffer_size(e.plan, &e.work) != rocfft_status_success) {
        rocfft_plan_destroy(e.plan);
        set_error("rocfft_plan_get_work_buffer_size failed");
        return AKB_E_FFT;
    }
    g_plans[key] = e;
    *out = e;
    return AKB_OK;
}

}  // namespace akb

using namespace akb;

extern "C" {

int64_t akb_psf_work_bytes(int ny, int nx, int pad, int batch) {
    if (ny <= 0 || nx <= 0 || pad < 1 || batch < 1) return -1;
    const PsfGeom g = psf_geom(ny, nx, pad);
    if (psf_line_ok(g, pad))  // G, peaks, rows, bounds, the select route's parts
        return psf_fast_bytes(g, batch) + 256 + 4 * psf_line_rows_bytes(g, batch) + psf_sel_bytes(g, batch);
    if (psf_fast_ok(g)) return psf_fast_bytes(g, batch);             // H (ey x px)
    PlanEntry e;
    if (get_plan(g.py, g.px, batch, &e) != AKB_OK) return -1;
    const int64_t field = (int64_t)batch * g.py * g.px * 16;
    const int64_t work = ((int64_t)e.work + 255) / 256 * 256;
    return field + work;
}

int akb_psf_f64(const double* opd, const double* amp, int ny, int nx, int pad, int batch,
                const double* lambdas, double dx, double dy, const double* hann_wy,
                const double* hann_wx, double hann_max, double* psf, double* efield_re_im,
                double* d_imax, const double* d_pitch, void* work, void* stream) {
    clear_error();
    AKB_REQUIRE(opd && lambdas && psf && d_imax && work, "null pointer");
    AKB_REQUIRE(ny > 0 && nx > 0 && pad >= 1, "bad pupil size / pad");
    AKB_REQUIRE(batch >= 1 && batch <= 8, "batch must be 1..8");
    AKB_REQUIRE((hann_wy == nullptr) == (hann_wx == nullptr), "hann needs both axes");
    const PsfGeom g = psf_geom(ny, nx, pad);
    hipStream_t s = (hipStream_t)stream;
    int st;
    if (psf_line_ok(g, pad)) {
        PsfLineArgs la{};
        la.opd = opd;
        la.amp = amp;
        la.wy = hann_wy;
        la.wx = hann_wx;
        la.wmax = hann_max;
        la.g = g;
        for (int b = 0; b < batch; ++b) la.kphase[b] = (2.0 * M_PI / lambdas[b]);
        char* tail = (char*)work + psf_fast_bytes(g, batch);
        la.G = (double2*)work;
        la.umax = (double*)tail;
        la.umax32 = (unsigned*)(tail + 64);
        la.cand_n = (int*)(tail + 128);
        la.rowmax32 = (float*)(tail + 256);
        la.cand = (int*)(tail + 256 + psf_line_rows_bytes(g, batch));
        la.ubmax = (double*)(tail + 160);
        la.ubound = (double*)(tail + 256 + 2 * psf_line_rows_bytes(g, batch));
        if ((st = get_twiddles(g.px, s, &la.Wx))) return st;
        if ((st = get_twiddles(g.py, s, &la.Wy))) return st;
        la.dA = dx * dy;
        la.pitch = d_pitch;
        la.psf = psf;
        la.efield = (double2*)efield_re_im;
        la.imax = d_imax;
        // the peak (same bits on every route): on planes of 2^24 points and up the row-bound
        // rounds (16384^2: 46 us of bounds + 2 x 12 us of rounds instead of a 0.91 ms fp64 pass or
        // the fp32 pass + re-run's 0.58 ms); below it the select route (pass 1 leaves the row
        // bounds and the centre samples, the peak pass transforms only the rows that can hold the
        // max: no launch beyond the three passes). AKB_PSF_PEAK = select / bound / f32 / f64 (every
        // row) forces a route.
        const char* pk = getenv("AKB_PSF_PEAK");
        const bool peak32 = pk && strcmp(pk, "f32") == 0;
        const bool bound = pk ? strcmp(pk, "bound") == 0 : (int64_t)g.py * g.px >= (1LL << 24);
        const bool select = psf_sel_ok(g) && (pk ? strcmp(pk, "select") == 0 : !bound);
        if (select) {
            char* sp = tail + 256 + 4 * psf_line_rows_bytes(g, batch);
            la.bpart = (double*)sp;
            la.spart = (double2*)(sp + ((int64_t)batch * g.nx2 * g.py * 8 + 255) / 256 * 256);
            la.npart = psf_line_pupil_wgs(g.ny2, pad, g.nx2);
            AKB_REQUIRE(la.npart >= 1 && la.npart <= g.nx2, "select route: pass-1 workgroups");
        }
        if ((st = psf_line_dispatch<kLinePupil>(g.ny2, pad, la, g.nx2, batch, s))) return st;
        if (bound) {
            k_psf_rowbound<<<dim3((g.py + 63) / 64, batch), 1024, 0, s>>>(la);
            if ((st = launch_status("k_psf_rowbound"))) return st;
            k_psf_bound_rows1<<<batch, 1024, 0, s>>>(la);
            if ((st = launch_status("k_psf_bound_rows1"))) return st;
            if ((st = psf_line_dispatch<kLinePeak>(g.nx2, pad, la, g.py, batch, s))) return st;
            k_psf_bound_rows2<<<batch, 1024, 0, s>>>(la);
            if ((st = launch_status("k_psf_bound_rows2"))) return st;
        } else if (peak32) {
            if ((st = psf_line_dispatch<kLinePeak32>(g.nx2, pad, la, g.py, batch, s))) return st;
            k_psf_peak_rows<<<batch, 1024, 0, s>>>(la, g.py / 4);
            if ((st = launch_status("k_psf_peak_rows"))) return st;
        } else {
            la.cand = nullptr;
        }
        if ((st = psf_line_dispatch<kLinePeak>(g.nx2, pad, la, g.py, batch, s))) return st;
        if (la.efield) return psf_line_dispatch<kLineWriteE>(g.nx2, pad, la, g.py, batch, s);
        return psf_line_dispatch<kLineWrite>(g.nx2, pad, la, g.py, batch, s);
    }
    if (psf_fast_ok(g)) {
        PsfFastArgs fa{};
        fa.opd = opd;
        fa.amp = amp;
        fa.wy = hann_wy;
        fa.wx = hann_wx;
        fa.wmax = hann_max;
        fa.g = g;
        for (int b = 0; b < batch; ++b) fa.kphase[b] = (2.0 * M_PI / lambdas[b]);
        fa.H = (double2*)work;
        fa.hT = g.ny2 >= 512;  // FftShape<N>::k3 of the column pass
        if ((st = get_twiddles(g.px, s, &fa.Wx))) return st;
        if ((st = get_twiddles(g.py, s, &fa.Wy))) return st;
        fa.dA = dx * dy;
        fa.pitch = d_pitch;
        fa.psf = psf;
        fa.efield = (double2*)efield_re_im;
        fa.imax = d_imax;
        if ((st = psf_rows_dispatch(g.nx2, fa, batch, s))) return st;
        return psf_cols_dispatch(g.ny2, fa, batch, s);
    }
    PlanEntry e;
    st = get_plan(g.py, g.px, batch, &e);
    if (st) return st;
    double2* field = (double2*)work;
    char* fft_work = (char*)work + (int64_t)batch * g.py * g.px * 16;

    PsfPupilArgs pa{};
    pa.opd = opd;
    pa.amp = amp;
    pa.wy = hann_wy;
    pa.wx = hann_wx;
    pa.wmax = hann_max;
    pa.g = g;
    for (int b = 0; b < batch; ++b) pa.kphase[b] = (2.0 * M_PI / lambdas[b]);
    pa.field = field;
    const int64_t total = (int64_t)g.py * g.px;
    const unsigned gx = (unsigned)((g.px + kBlock - 1) / kBlock);
    // rows per workgroup: ~1k workgroups in all, so the per-workgroup peak atomics stay few
    const unsigned gy = (unsigned)(g.py < 128 ? g.py : 128);
    k_psf_pupil<<<dim3(gx, gy, batch), kBlock, 0, s>>>(pa);
    if ((st = launch_status("k_psf_pupil"))) return st;

    rocfft_execution_info info = nullptr;
    if (rocfft_execution_info_create(&info) != rocfft_status_success) {
        set_error("rocfft_execution_info_create failed");
        return AKB_E_FFT;
    }
    rocfft_execution_info_set_stream(info, (void*)s);
    if (e.work) rocfft_execution_info_set_work_buffer(info, fft_work, e.work);
    void* bufs[1] = {field};
    rocfft_status fs = rocfft_execute(e.plan, bufs, nullptr, info);
    rocfft_execution_info_destroy(info);
    if (fs != rocfft_status_success) {
        set_error("rocfft_execute failed: %d", (int)fs);
        return AKB_E_FFT;
    }

    AKB_HIP_CHECK(hipMemsetAsync(d_imax, 0, sizeof(double) * batch, s));
    PsfIntenArgs ia{};
    ia.field = field;
    ia.g = g;
    ia.dA = dx * dy;
    ia.pitch = d_pitch;
    ia.psf = psf;
    ia.efield = (double2*)efield_re_im;
    ia.imax = d_imax;
    k_psf_inten<<<dim3(gx, gy, batch), kBlock, 0, s>>>(ia);
    if ((st = launch_status("k_psf_inten"))) return st;
    k_psf_norm<<<dim3(grid_for(total, 1, kStreamGridCap), 1, batch), kBlock, 0, s>>>(psf, (double2*)efield_re_im, d_imax, total);
    return launch_status("k_psf_norm");
}

void akb_psf_release_plans(void) {
    {
        std::lock_guard<std::mutex> lk(g_plan_mu);
        for (auto& kv : g_plans) rocfft_plan_destroy(kv.second.plan);
        g_plans.clear();
        if (g_rocfft_ready) {  // rocFFT's own caches too, before the HIP runtime's teardown
            rocfft_cleanup();
            g_rocfft_ready = false;
        }
    }
    std::lock_guard<std::mutex> lk(g_tw_mu);
    for (auto& kv : g_tw) (void)hipFree(kv.second);
    g_tw.clear();
}

}  // extern "C"

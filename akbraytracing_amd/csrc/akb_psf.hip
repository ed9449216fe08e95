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
#include <rocfft/rocfft.h>

#include <map>
#include <mutex>
#include <tuple>

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
    // which reproduces numpy's NaN-propagating max
    atomicMax((unsigned long long*)addr, (unsigned long long)__double_as_longlong(v));
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
    PlanEntry e;
    int st = get_plan(g.py, g.px, batch, &e);
    if (st) return st;
    hipStream_t s = (hipStream_t)stream;
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
    std::lock_guard<std::mutex> lk(g_plan_mu);
    for (auto& kv : g_plans) rocfft_plan_destroy(kv.second.plan);
    g_plans.clear();
}

}  // extern "C"

// psf_calc's pupil preparation for gfx950 (AKB_raytrace_20250312.py:1121-1188): the rotation
// estimate's per-column first valid row, and rotate_with_nan(order=3) — scipy.ndimage.rotate
// (reshape=False, mode 'constant') of the NaN-filled map and of its finite mask, divided, NaN
// where the rotated mask < 0.5.
//
// scipy's order-3 rotate is a cubic B-spline prefilter along each axis followed by a 4 x 4
// B-spline sum at each output pixel's source point (oracle/psfcalc.py states the algorithm and
// its boundary rules). The maps are small (65^2 .. 1k^2): one thread per line for the recursive
// prefilter, one thread per output pixel for the interpolation, both arrays at once.
#include "akb_common.h"

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
__global__ void k_spline_lines(double* __restrict__ coef, int ny, int nx, int axis) {
    // blockIdx.y: which array (map, mask); one thread per line
    const int line = blockIdx.x * blockDim.x + threadIdx.x;
    const int nlines = axis == 0 ? nx : ny;
    if (line >= nlines) return;
    double* base = coef + (int64_t)blockIdx.y * ny * nx;
    const int n = axis == 0 ? ny : nx;
    const int64_t s = axis == 0 ? nx : 1;
    double* c = base + (axis == 0 ? line : (int64_t)line * nx);
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

__global__ void k_rotate_cubic(RotArgs a) {
    const int64_t total = (int64_t)a.ny * a.nx;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < total; k += (int64_t)gridDim.x * blockDim.x) {
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

}  // extern "C"

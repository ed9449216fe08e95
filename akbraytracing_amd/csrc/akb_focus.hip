// Focus evaluation for gfx950: the tail of plot_result_debug's 'test' mode and the spot sizes
// auto_focus_NA minimises (AKB_raytrace_20250312.py:2842-2847, :3565-3601, :12785-12786).
//
// Input: rays already traced through the mirrors (exit direction and last hit, (3, n) per
// system), one or more detector planes x = -j per system, and the tilt rotation of each system
// (R_y, R_z of rotate_vectors, formed by the host from np.nanmean(np.arctan(...)) of the same
// directions) or none (option_tilt=False). Per (system, plane) one workgroup:
//   det0  = plane(j; dir, pt)                                        (:2842-2845)
//   focus = np.mean(det0, axis=1)                                    (:3591)
//   dir'  = R_y @ (R_z @ dir), pt' = R_y @ (R_z @ (pt - focus)) + focus (:3590-3592, dgemm order)
//   det   = plane(j; dir', pt')                                      (:3593-3596)
//   out   = np.std(det[2]), np.std(det[1])                           (:12785-12786)
// Every mean and sum is numpy's pairwise order (akb_pairwise.h), so the sizes - and the argmin
// auto_focus_NA takes over them - are the reference's to the bit. A sweep of auto_focus_NA is one
// system against 100 planes: 100 workgroups reading the same L2-resident rays; the per-ray rows
// the two-pass reductions need live in a per-workgroup scratch slab (L2-resident at these sizes).
#include "akb_pairwise.h"

namespace akb {

constexpr int kFocBlock = 256;  // 4 waves: up to 3 row sums side by side
constexpr int kFocRows = 5;

struct FocusArgs {
    const double* dir;  // system s: rows at dir + s * sys_ld + k * n
    const double* pt;
    int64_t n, sys_ld;
    int P;
    const double* plane_j;  // (S * P): plane x = -j (coeffs_det[9] = j, g = 1)
    const double* rot;      // (S, 18): R_y then R_z, row-major; NULL: no tilt
    double* out;            // (S * P, 2): np.std(det z), np.std(det y)
    double* det_out;        // (S * P, 3, n) or NULL
    double* dir_out;        // (S * P, 3, n) or NULL: the (tilted) directions, the 'test' return's angle
    double* work;           // (S * P, kFocRows, n)
};

// np.sum of a[0..n), n >= 1, by one wave: each 8192-element buffer pairwise, buffers added left
// to right
__device__ static double wave_np_sum(PwTree& T, const double* a, int64_t n) {
    double acc = 0.0;
    for (int64_t b = 0; b < n; b += 8192) {
        const int len = (int)(n - b < 8192 ? n - b : 8192);
        const double v = pw_tree_wave(T, a + b, len);
        acc = b == 0 ? v : acc + v;
    }
    return acc;
}

__global__ void __launch_bounds__(kFocBlock) k_focus_eval(FocusArgs A) {
    __shared__ PwTree T[3];
    __shared__ double red[8];
    const int64_t sp = blockIdx.x;
    const int64_t s = sp / A.P;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t n = A.n;
    const double* D = A.dir + s * A.sys_ld;
    const double* Q = A.pt + s * A.sys_ld;
    double* W = A.work + sp * kFocRows * n;
    const double j = A.plane_j[sp];
    const bool tilt = A.rot != nullptr;
    double* det = A.det_out ? A.det_out + sp * 3 * n : nullptr;
    double* ang = A.dir_out ? A.dir_out + sp * 3 * n : nullptr;

    // detector hits of the traced rays
    for (int64_t i = threadIdx.x; i < n; i += kFocBlock) {
        const double l = D[i], m = D[n + i], nn = D[2 * n + i];
        double x, y, z;
        plane_hit(1.0, 0.0, 0.0, j, l, m, nn, Q[i], Q[n + i], Q[2 * n + i], x, y, z);
        W[i] = x;
        W[n + i] = y;
        W[2 * n + i] = z;
        if (!tilt && det) {
            det[i] = x;
            det[n + i] = y;
            det[2 * n + i] = z;
        }
        if (!tilt && ang) {
            ang[i] = l;
            ang[n + i] = m;
            ang[2 * n + i] = nn;
        }
    }
    __syncthreads();
    int ry = 1, rz = 2;
    if (tilt) {
        if (w < 3) {
            const double sum = wave_np_sum(T[w], W + w * n, n);
            if (lane == 0) red[w] = sum / (double)n;  // np.mean: true_divide(sum, n)
        }
        __syncthreads();
        const double cx = red[0], cy = red[1], cz = red[2];
        Mat3 Ry, Rz;
        const double* R = A.rot + s * 18;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            Ry.m[k] = R[k];
            Rz.m[k] = R[9 + k];
        }
        for (int64_t i = threadIdx.x; i < n; i += kFocBlock) {
            double ax, ay, az, l, m, nn, px, py, pz;
            matvec(Rz, D[i], D[n + i], D[2 * n + i], ax, ay, az);
            matvec(Ry, ax, ay, az, l, m, nn);
            matvec(Rz, Q[i] - cx, Q[n + i] - cy, Q[2 * n + i] - cz, ax, ay, az);
            matvec(Ry, ax, ay, az, px, py, pz);
            px = px + cx;
            py = py + cy;
            pz = pz + cz;
            double x, y, z;
            plane_hit(1.0, 0.0, 0.0, j, l, m, nn, px, py, pz, x, y, z);
            W[3 * n + i] = y;
            W[4 * n + i] = z;
            if (det) {
                det[i] = x;
                det[n + i] = y;
                det[2 * n + i] = z;
            }
            if (ang) {
                ang[i] = l;
                ang[n + i] = m;
                ang[2 * n + i] = nn;
            }
        }
        ry = 3;
        rz = 4;
        __syncthreads();
    }
    // np.std: mean = sum / n, then the sum of squared deviations / n, sqrt
    if (w < 2) {
        const double sum = wave_np_sum(T[w], W + (w == 0 ? rz : ry) * n, n);
        if (lane == 0) red[4 + w] = sum / (double)n;
    }
    __syncthreads();
    const double mz = red[4], my = red[5];
    for (int64_t i = threadIdx.x; i < n; i += kFocBlock) {
        const double dz = W[rz * n + i] - mz, dy = W[ry * n + i] - my;
        W[i] = dz * dz;  // rows 0 and 1 are free by now (each thread rewrites only its own rays)
        W[n + i] = dy * dy;
    }
    __syncthreads();
    if (w < 2) {
        const double ss = wave_np_sum(T[w], W + w * n, n);
        if (lane == 0) A.out[sp * 2 + w] = sqrt(ss / (double)n);
    }
}

}  // namespace akb

using namespace akb;

extern "C" {

int64_t akb_focus_eval_work_bytes(int n_sys, int n_planes, int64_t n) {
    if (n_sys <= 0 || n_planes <= 0 || n <= 0) return 0;
    return (int64_t)n_sys * n_planes * kFocRows * n * 8;
}

int akb_focus_eval_f64(const double* dir, const double* pt, int64_t n, int64_t sys_ld, int n_sys, int n_planes,
                       const double* d_plane_j, const double* d_rot, double* d_std, double* det_out, double* dir_out,
                       void* work, void* stream) {
    clear_error();
    AKB_REQUIRE(dir && pt && d_plane_j && d_std && work, "null pointer");
    AKB_REQUIRE(n >= 1 && n < (1LL << 31), "n out of range");
    AKB_REQUIRE(n_sys >= 1 && n_planes >= 1 && (int64_t)n_sys * n_planes < (1LL << 31), "bad system / plane count");
    AKB_REQUIRE(sys_ld >= 3 * n || n_sys == 1, "system blocks overlap (sys_ld < 3 n)");
    FocusArgs a{dir, pt, n, sys_ld, n_planes, d_plane_j, d_rot, d_std, det_out, dir_out, (double*)work};
    const unsigned g = (unsigned)((int64_t)n_sys * n_planes);
    k_focus_eval<<<g, kFocBlock, 0, (hipStream_t)stream>>>(a);
    return launch_status("k_focus_eval");
}

}  // extern "C"

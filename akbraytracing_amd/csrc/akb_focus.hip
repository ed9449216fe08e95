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

// ---------------------------------------------------------------------------------------------
// compare_sep's plane searches (AKB_raytrace_20250312.py:9174-9560). A search minimises
//   f(a) = sqrt(np.std(det_z)**2 + np.std(det_y)**2),  det = plane x = -a hit by a ray subset
// (:9233-9256) by optimize_min_index (:9174-9217): 100 points of np.linspace(x_min, x_max), the
// first argmin (a NaN wins, as np.argmin), the range shrunk by 0.1 about it, until narrower than
// 1e-13. Every step depends on the last, but the 100 points of a step are independent: one
// workgroup per search, one lane per point, the whole coarse-to-fine loop inside the kernel (one
// launch for compare_sep's twenty searches instead of ~26000 numpy plane intersections). A lane
// sums its point's rows in numpy's pairwise order without storing them: the hit of ray i is
// recomputed in each of np.std's two passes (same inputs, same bits).

constexpr int kSepBlock = 128;  // >= the reference's 100 points per step
constexpr int kSepMax = 32;     // searches per launch (compare_sep runs 20)

struct SepArgs {
    const double* dir;  // (3, ld) exit directions
    const double* pt;   // (3, ld) last hits
    int64_t ld;
    int64_t start[kSepMax], step[kSepMax], count[kSepMax];  // subset of search q: start + i * step
    double x_min, x_max, shrink, tol;
    int num, max_attempts;
    double* out;  // (Q, 4): best_x, min_y, the last x evaluated, the final range width
};

struct Sum2 {
    double a, b;
};

// hit of subset element i on plane x = -a: (y, z), or (y - my)^2, (z - mz)^2 in pass 2
struct SepRow {
    const double* dir;
    const double* pt;
    int64_t ld, start, step;
    double j, my, mz;
    bool sq;
    __device__ Sum2 operator()(int64_t i) const {
        const int64_t r = start + i * step;
        double x, y, z;
        plane_hit(1.0, 0.0, 0.0, j, dir[r], dir[ld + r], dir[2 * ld + r], pt[r], pt[ld + r], pt[2 * ld + r], x, y, z);
        if (!sq) return {y, z};
        const double dy = y - my, dz = z - mz;
        return {dy * dy, dz * dz};
    }
};

__device__ static Sum2 sep_leaf(const SepRow& f, int64_t o, int n) {
    if (n < 8) {
        Sum2 s{0.0, 0.0};
        for (int i = 0; i < n; ++i) {
            const Sum2 v = f(o + i);
            s.a = s.a + v.a;
            s.b = s.b + v.b;
        }
        return s;
    }
    double ra[8], rb[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const Sum2 v = f(o + k);
        ra[k] = v.a;
        rb[k] = v.b;
    }
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const Sum2 v = f(o + i + k);
            ra[k] = ra[k] + v.a;
            rb[k] = rb[k] + v.b;
        }
    }
    Sum2 s{((ra[0] + ra[1]) + (ra[2] + ra[3])) + ((ra[4] + ra[5]) + (ra[6] + ra[7])),
           ((rb[0] + rb[1]) + (rb[2] + rb[3])) + ((rb[4] + rb[5]) + (rb[6] + rb[7]))};
    for (; i < n; ++i) {
        const Sum2 v = f(o + i);
        s.a = s.a + v.a;
        s.b = s.b + v.b;
    }
    return s;
}

// numpy's pairwise_sum over one buffer (n <= 8192: six splits reach a <= 128 leaf); one function
// per depth, not inlined, so the tree costs seven small functions instead of 64 leaf copies
template <int D>
__device__ __attribute__((noinline)) Sum2 sep_pw(const SepRow& f, int64_t o, int n) {
    if constexpr (D == 0) {
        return sep_leaf(f, o, n);
    } else {
        if (n <= kPwLeaf) return sep_leaf(f, o, n);
        const int n2 = pw_split(n);
        const Sum2 l = sep_pw<D - 1>(f, o, n2);
        const Sum2 r = sep_pw<D - 1>(f, o + n2, n - n2);
        return {l.a + r.a, l.b + r.b};
    }
}

// np.sum over count elements: 8192-element buffers pairwise, added left to right
__device__ static Sum2 sep_sum(const SepRow& f, int64_t count) {
    Sum2 acc{0.0, 0.0};
    for (int64_t b = 0; b < count; b += 8192) {
        const int len = (int)(count - b < 8192 ? count - b : 8192);
        const Sum2 v = sep_pw<6>(f, b, len);
        acc = b == 0 ? v : Sum2{acc.a + v.a, acc.b + v.b};
    }
    return acc;
}

__global__ void __launch_bounds__(kSepBlock) k_sep_search(SepArgs A) {
    __shared__ double xs[kSepBlock], ys[kSepBlock];
    const int q = blockIdx.x, t = threadIdx.x;
    const int64_t cnt = A.count[q];
    const int num = A.num;
    double x_min = A.x_min, x_max = A.x_max;
    double best_x = 0.0, min_y = 0.0, last_x = 0.0;
    for (int attempt = 0; attempt < A.max_attempts; ++attempt) {
        // np.linspace(x_min, x_max, num): i * step + start, the last point = stop exactly
        const double div = (double)(num - 1);
        const double delta = x_max - x_min;
        const double step = delta / div;
        if (t < num) {
            double x = step == 0.0 ? ((double)t / div) * delta : (double)t * step;
            x = x + x_min;
            if (t == num - 1 && num > 1) x = x_max;
            double y;
            if (cnt == 0) {
                y = __builtin_nan("");  // np.std of an empty subset
            } else {
                SepRow f{A.dir, A.pt, A.ld, A.start[q], A.step[q], x, 0.0, 0.0, false};
                const Sum2 s = sep_sum(f, cnt);
                f.my = s.a / (double)cnt;  // np.mean: true_divide(sum, n)
                f.mz = s.b / (double)cnt;
                f.sq = true;
                const Sum2 ss = sep_sum(f, cnt);
                const double sh = sqrt(ss.a / (double)cnt), sv = sqrt(ss.b / (double)cnt);
                y = sqrt(sv * sv + sh * sh);  // np.float64 ** 2 is the rounded square
            }
            xs[t] = x;
            ys[t] = y;
        }
        __syncthreads();
        // np.argmin: the first NaN, else the first minimum (every lane, same answer)
        int bi = 0;
        double by = ys[0];
        for (int k = 1; k < num && by == by; ++k) {
            const double v = ys[k];
            if (v < by || v != v) {
                by = v;
                bi = k;
            }
        }
        best_x = xs[bi];
        min_y = by;
        last_x = xs[num - 1];
        const double delta_x = (x_max - x_min) * A.shrink;
        x_min = best_x - delta_x / 2.0;
        x_max = best_x + delta_x / 2.0;
        __syncthreads();  // xs / ys are rewritten by the next step
        if ((x_max - x_min) < A.tol && x_max - x_min > 1e-16) break;
    }
    if (t == 0) {
        A.out[q * 4 + 0] = best_x;
        A.out[q * 4 + 1] = min_y;
        A.out[q * 4 + 2] = last_x;
        A.out[q * 4 + 3] = x_max - x_min;
    }
}

}  // namespace akb

using namespace akb;

extern "C" {

int akb_sep_search_f64(const double* dir, const double* pt, int64_t ld, int64_t n, int n_search,
                       const int64_t* h_start, const int64_t* h_step, const int64_t* h_count, double x_min,
                       double x_max, int num_steps, int max_attempts, double shrink, double tol, double* d_out,
                       void* stream) {
    clear_error();
    AKB_REQUIRE(dir && pt && h_start && h_step && h_count && d_out, "null pointer");
    AKB_REQUIRE(n >= 0 && ld >= n, "bad row length");
    AKB_REQUIRE(n_search >= 1 && n_search <= kSepMax, "1 <= n_search <= 32");
    AKB_REQUIRE(num_steps >= 2 && num_steps <= kSepBlock, "2 <= num_steps <= 128");
    AKB_REQUIRE(max_attempts >= 1, "max_attempts >= 1");
    SepArgs a{};
    a.dir = dir;
    a.pt = pt;
    a.ld = ld;
    for (int q = 0; q < n_search; ++q) {
        const int64_t c = h_count[q], s0 = h_start[q], st = h_step[q];
        AKB_REQUIRE(c >= 0, "negative subset size");
        if (c > 0) {
            const int64_t last = s0 + (c - 1) * st;
            AKB_REQUIRE(s0 >= 0 && s0 < n && last >= 0 && last < n, "subset index out of range");
        }
        a.start[q] = s0;
        a.step[q] = st;
        a.count[q] = c;
    }
    a.x_min = x_min;
    a.x_max = x_max;
    a.shrink = shrink;
    a.tol = tol;
    a.num = num_steps;
    a.max_attempts = max_attempts;
    a.out = d_out;
    k_sep_search<<<n_search, kSepBlock, 0, (hipStream_t)stream>>>(a);
    return launch_status("k_sep_search");
}

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

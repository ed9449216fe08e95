// Ray-trace kernels for gfx950: the reference's numpy primitives (one kernel each, the drop-in
// stage API) and the fused mirror chain (device-resident API used by the AKB/KB pipelines).
//
// Layout: every ray quantity is struct-of-arrays float64, (3, ld) C-order, exactly the layout
// of the reference's (3, N) numpy arrays (AKB_raytrace_20250312.py:2694-2717), so a wave's 64
// lanes read 64 consecutive doubles of one row: fully coalesced 512-B segments per row.
// Mirror coefficients travel in the kernel argument segment and are read with scalar loads
// (wave-uniform, SGPR-resident), so the per-ray stream is only positions and directions.
#include <math.h>

#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "akb_common.h"
#include "akb_pairwise.h"
#include "akb_sincos.h"

namespace akb {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
}
void clear_error() { g_last_error.clear(); }

// ----------------------------------------------------------------------------------------------
// stage kernels
// ----------------------------------------------------------------------------------------------

__global__ void __launch_bounds__(kBlock) k_isect(Quadric Q, V3In dir, V3In org, int negative,
                                                  int64_t n, V3Out out, int32_t* flags) {
    int fl = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        double x, y, z;
        const bool ok = quadric_hit(Q, dir.x(i), dir.y(i), dir.z(i), org.x(i), org.y(i), org.z(i),
                                    negative != 0, x, y, z);
        if (!ok) fl |= AKB_FLAG_MISS;
        out.store(i, x, y, z);
    }
    if (fl) atomicOr(flags, fl);
}

__global__ void __launch_bounds__(kBlock) k_normal(Quadric Q, V3In pt, int64_t n, V3Out out,
                                                   int normalize, int32_t* flags) {
    int fl = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        double nx, ny, nz;
        quadric_grad(Q, pt.x(i), pt.y(i), pt.z(i), nx, ny, nz);
        if (normalize) {
            const double s = norm3(nx, ny, nz);
            if (s == 0.0) fl |= AKB_FLAG_ZERO_NORMAL;
            out.store(i, nx / s, ny / s, nz / s);
        } else {
            out.store(i, nx, ny, nz);
        }
    }
    if (fl) atomicOr(flags, fl);
}

__global__ void __launch_bounds__(kBlock) k_reflect(V3In dir, V3In nrm, int64_t n, V3Out out,
                                                    int normalize, int32_t* flags) {
    int fl = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        double rx, ry, rz;
        reflect_raw(dir.x(i), dir.y(i), dir.z(i), nrm.x(i), nrm.y(i), nrm.z(i), rx, ry, rz);
        if (normalize) {
            const double s = norm3(rx, ry, rz);
            if (s == 0.0) fl |= AKB_FLAG_ZERO_REFLECT;
            out.store(i, rx / s, ry / s, rz / s);
        } else {
            out.store(i, rx, ry, rz);
        }
    }
    if (fl) atomicOr(flags, fl);
}

__global__ void __launch_bounds__(kBlock) k_normalize(V3In v, int64_t n, V3Out out, int32_t* flags) {
    int fl = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double x = v.x(i), y = v.y(i), z = v.z(i);
        const double s = norm3(x, y, z);
        if (s == 0.0) fl |= AKB_FLAG_ZERO_DIR;
        out.store(i, x / s, y / s, z / s);
    }
    if (fl) atomicOr(flags, fl);
}

__global__ void __launch_bounds__(kBlock) k_plane(double g, double h, double ii, double j, V3In dir,
                                                  V3In org, int64_t n, V3Out out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        double x, y, z;
        plane_hit(g, h, ii, j, dir.x(i), dir.y(i), dir.z(i), org.x(i), org.y(i), org.z(i), x, y, z);
        out.store(i, x, y, z);
    }
}

__global__ void __launch_bounds__(kBlock) k_seglen(V3In a, V3In b, int64_t n, double* out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        out[i] = norm3(b.x(i) - a.x(i), b.y(i) - a.y(i), b.z(i) - a.z(i));
    }
}

__global__ void __launch_bounds__(kBlock) k_rotate(Mat3 Ry, Mat3 Rz, double cx, double cy, double cz,
                                                   int shift, V3In v, int64_t n, V3Out out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        double x = v.x(i), y = v.y(i), z = v.z(i);
        if (shift) {
            x = x - cx;
            y = y - cy;
            z = z - cz;
        }
        double ax, ay, az, bx, by, bz;
        matvec(Rz, x, y, z, ax, ay, az);
        matvec(Ry, ax, ay, az, bx, by, bz);
        if (shift) {
            bx = bx + cx;
            by = by + cy;
            bz = bz + cz;
        }
        out.store(i, bx, by, bz);
    }
}

__global__ void k_fill_nan(double* out, int64_t ld, int rows, int64_t n) {
    const double qnan = __builtin_nan("");
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        for (int r = 0; r < rows; ++r) out[r * ld + i] = qnan;
    }
}

// ----------------------------------------------------------------------------------------------
// focus sweeps (find_defocus, ref AKB_raytrace_20250312.py:9086-9170): one set of rays against P
// detector planes x = -j_p at once. Pass A writes each plane's hit y and z rows; pass B, given the
// numpy-order sums of pass A, writes (y - mean)^2 and (z - mean)^2 — np.std's two passes, the
// sums in between by akb_pairwise_sum_f64 so the result is numpy's to the bit.
// ----------------------------------------------------------------------------------------------

__global__ void __launch_bounds__(kBlock) k_plane_sweep(const double* __restrict__ dir, const double* __restrict__ pt,
                                                        int64_t ld, const int64_t* __restrict__ subset, int64_t m,
                                                        const double* __restrict__ plane_j, int P,
                                                        const double* __restrict__ sums, double n_div,
                                                        double* __restrict__ rows) {
    const int p = blockIdx.y;
    const double j = plane_j[p];
    double my = 0.0, mz = 0.0;
    if (sums) {  // np.mean: true_divide(sum, n)
        my = sums[2 * p] / n_div;
        mz = sums[2 * p + 1] / n_div;
    }
    double* ry = rows + (int64_t)(2 * p) * m;
    double* rz = ry + m;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = subset ? subset[k] : k;
        double x, y, z;
        plane_hit(1.0, 0.0, 0.0, j, dir[i], dir[ld + i], dir[2 * ld + i], pt[i], pt[ld + i], pt[2 * ld + i], x, y, z);
        (void)x;
        if (sums) {
            const double dy = y - my, dz = z - mz;
            ry[k] = dy * dy;
            rz[k] = dz * dz;
        } else {
            ry[k] = y;
            rz[k] = z;
        }
    }
}

// The same sweep with np.std's two sums fused: each workgroup loads a 256-ray segment once and,
// plane after plane, hands the segment's y / z (pass A) or squared deviations (pass B) to a leaf
// sink of 2P quantities (plane p -> quantities 2p, 2p + 1). Nothing per plane reaches HBM but the
// leaf sums, and the rays are read once per pass instead of once per plane.
constexpr int kSweepGroup = 8;  // planes per leaf reduction round (16 quantities: every thread busy)

__global__ void __launch_bounds__(kBlock) k_plane_sweep_sink(const double* __restrict__ dir,
                                                             const double* __restrict__ pt, int64_t ld,
                                                             const int64_t* __restrict__ subset, int64_t m,
                                                             const double* __restrict__ plane_j, int P,
                                                             const double* __restrict__ sums, double n_div,
                                                             akb_leaf_sink sink) {
    __shared__ LeafLds<2 * kSweepGroup> L;
    extern __shared__ double mean[];  // pass B: the 2P means, divided once per workgroup
    if (sums) {
        for (int q = threadIdx.x; q < 2 * P; q += blockDim.x) mean[q] = sums[q] / n_div;  // np.mean: sum / n
        __syncthreads();
    }
    const int64_t nseg = (m + kLeafSeg - 1) / kLeafSeg;
    const int64_t nleaves = (sink.n / kNpBuf) * kNpBuf / 128;
    for (int64_t seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
        const int64_t k = seg * kLeafSeg + threadIdx.x;
        const bool valid = k < m;
        double l = 0.0, mm = 0.0, nn = 0.0, px = 0.0, py = 0.0, pz = 0.0;
        if (valid) {
            const int64_t i = subset ? subset[k] : k;
            l = dir[i];
            mm = dir[ld + i];
            nn = dir[2 * ld + i];
            px = pt[i];
            py = pt[ld + i];
            pz = pt[2 * ld + i];
        }
        // plane_hit's denominator (1 l + 0 m + 0 n) is the same for every plane: one IEEE
        // reciprocal, then each plane's quotient by the shared-reciprocal correction (RN(x / s)
        // exactly, div_shared); a zero / non-finite / tiny denominator takes the plain division
        const double den = 1.0 * l + 0.0 * mm + 0.0 * nn;
        const double inv = 1.0 / den;
        const bool shared = fabs(den) >= 0x1p-900 && fabs(den) <= 0x1p+900;
        for (int p0 = 0; p0 < P; p0 += kSweepGroup) {
            double v[2 * kSweepGroup];
#pragma unroll
            for (int g = 0; g < kSweepGroup; ++g) {
                const int p = p0 + g;
                v[2 * g] = 0.0;
                v[2 * g + 1] = 0.0;
                if (valid && p < P) {
                    const double num = -(1.0 * px + 0.0 * py + 0.0 * pz + plane_j[p]);
                    const double an = fabs(num);
                    const bool ok = shared && (num == 0.0 || (an >= 0x1p-900 && an <= 0x1p+900));
                    const double t = ok ? div_shared(num, den, inv) : num / den;
                    const double y = t * mm + py;
                    const double z = t * nn + pz;
                    if (sums) {
                        const double dy = y - mean[2 * p], dz = z - mean[2 * p + 1];
                        v[2 * g] = dy * dy;
                        v[2 * g + 1] = dz * dz;
                    } else {
                        v[2 * g] = y;
                        v[2 * g + 1] = z;
                    }
                }
            }
            // quantities 2 p0 .. 2 p0 + 15 (the sink is padded to a multiple of 16)
            akb_leaf_sink S = sink;
            S.leaf_sum += (int64_t)(2 * p0) * nleaves;
            S.leaf_cnt += (int64_t)(2 * p0) * nleaves;
            S.tail += (int64_t)(2 * p0) * kNpBuf;
            leaf_sink_segment<2 * kSweepGroup>(S, L, seg * kLeafSeg, v, valid);
        }
    }
}

// ----------------------------------------------------------------------------------------------
// calc_dS (ref AKB_raytrace_20250312.py:13418-13473): the area element of each point of a (V, H)
// grid of mirror points = half the summed |cross| of its four neighbour triangles (right-up,
// up-left, left-down, down-right); border points take the value of the nearest interior point
// (the reference's edge and corner copies are exactly that clamp).
// ----------------------------------------------------------------------------------------------

__device__ __forceinline__ double tri_area(double x0, double y0, double z0, double x1, double y1, double z1,
                                           double x2, double y2, double z2) {
    const double ax = x1 - x0, ay = y1 - y0, az = z1 - z0;
    const double bx = x2 - x0, by = y2 - y0, bz = z2 - z0;
    const double cx = ay * bz - az * by;  // np.cross
    const double cy = az * bx - ax * bz;
    const double cz = ax * by - ay * bx;
    // np.linalg.norm of a 3-vector goes to BLAS ddot: x0 x0, then fma(x1, x1, .), fma(x2, x2, .)
    return sqrt(__builtin_fma(cz, cz, __builtin_fma(cy, cy, cx * cx))) / 2.0;
}

__global__ void __launch_bounds__(kBlock) k_calc_ds(const double* __restrict__ pts, int64_t ld, int V, int H,
                                                    double* __restrict__ out) {
    const int64_t total = (int64_t)V * H;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < total; k += (int64_t)gridDim.x * blockDim.x) {
        const int i0 = (int)(k / H), j0 = (int)(k - (int64_t)i0 * H);
        const int i = i0 < 1 ? 1 : (i0 > V - 2 ? V - 2 : i0);
        const int j = j0 < 1 ? 1 : (j0 > H - 2 ? H - 2 : j0);
        auto P = [&](int a, int b, double& x, double& y, double& z) {
            const int64_t c = (int64_t)a * H + b;
            x = pts[c];
            y = pts[ld + c];
            z = pts[2 * ld + c];
        };
        double px, py, pz, rx, ry, rz, ux, uy, uz, lx, ly, lz, dx, dy, dz;
        P(i, j, px, py, pz);
        P(i, j + 1, rx, ry, rz);
        P(i, j - 1, lx, ly, lz);
        P(i - 1, j, ux, uy, uz);
        P(i + 1, j, dx, dy, dz);
        double s = 0.0;
        s = s + tri_area(px, py, pz, rx, ry, rz, ux, uy, uz);
        s = s + tri_area(px, py, pz, ux, uy, uz, lx, ly, lz);
        s = s + tri_area(px, py, pz, lx, ly, lz, dx, dy, dz);
        s = s + tri_area(px, py, pz, dx, dy, dz, rx, ry, rz);
        out[k] = s;
    }
}

// tilt correction inputs (defined ahead of the chain: the fused pass-1 + tilt kernel loads them
// while it traces)
struct TiltArgs {
    Mat3 Ry, Rz;
    double c[3];
    const double* params;  // non-NULL: Ry, Rz, c from akb_tilt_params_f64's device block
    double d1[4], d2[4];
    const double* dir;
    const double* pt;
    const double* opl;
    int64_t ld, n;
    double* dir_rot;
    double* pt_rot;
    double* det1;
    double* det2;
    double* total1;
    double* total2;
    akb_leaf_sink sink;
};

// one ray's inputs (direction, last hit, OPL), loaded ahead of the arithmetic
struct TiltIn {
    double d[3], p[3], o;
};

// the same with the OPL row known to be present (no load under a branch: the fused kernel's wait
// counts then stay exact across both paths), for ray i0 + off / 8 of a segment starting at the
// wave-uniform i0: scalar row bases plus one 32-bit lane offset
__device__ __forceinline__ void tilt_load_seg(const TiltArgs& a, int64_t i0, uint32_t off, TiltIn& t) {
    const double* d = a.dir + i0;
    const double* p = a.pt + i0;
    t.d[0] = ld_off(d, off);
    t.d[1] = ld_off(d + a.ld, off);
    t.d[2] = ld_off(d + 2 * a.ld, off);
    t.p[0] = ld_off(p, off);
    t.p[1] = ld_off(p + a.ld, off);
    t.p[2] = ld_off(p + 2 * a.ld, off);
    t.o = ld_off(a.opl + i0, off);
}

__device__ __forceinline__ void tilt_load(const TiltArgs& a, int64_t i, TiltIn& t) {
    t.d[0] = a.dir[i];
    t.d[1] = a.dir[a.ld + i];
    t.d[2] = a.dir[2 * a.ld + i];
    t.p[0] = a.pt[i];
    t.p[1] = a.pt[a.ld + i];
    t.p[2] = a.pt[2 * a.ld + i];
    t.o = a.opl ? a.opl[i] : 0.0;
}

// ----------------------------------------------------------------------------------------------
// fused chain: K mirrors (+ detector plane + OPL) per ray, all intermediate state in registers
// ----------------------------------------------------------------------------------------------

// a chain mirror: the quadric plus its doubled square coefficients (2a, 2b, 2c: exact, formed on the
// host so the per-ray code does not recompute wave-uniform values on the vector ALU)
// sgn: +1.0, or -1.0 for a mirror traced with the minus root (negative=True): the root's sign as a
// factor, sD * sgn, instead of both roots and a per-lane select (x + (-y) is x - y exactly)
struct CMirror {
    double a, b, c, d, e, f, g, h, i, j, a2, b2, c2, sgn;
};

// mirror kinds: 0 general, 1 y-free (b = d = f = h = 0, h = +0.0), 2 z-free (c = e = f = i = 0, i = +0.0)
constexpr int kKindGeneral = 0, kKindYFree = 1, kKindZFree = 2;

struct ChainArgs {
    int K;
    int kind[AKB_MAX_MIRRORS];
    CMirror q[AKB_MAX_MIRRORS];
    double det[4];
    const double* dir;
    int64_t dir_ld, dir_inc;
    const double* tan_h;
    const double* tan_v;
    uint32_t n_h;
    uint32_t n_v;
    uint32_t div_mul;  // Granlund-Montgomery magic for g / n_h with 32-bit g (see div_magic)
    uint32_t div_shift;
    int64_t g0;        // global flat index of ray 0 of this launch
    int64_t g_stride;  // flat-index step between consecutive rays (1; n_h walks a grid column)
    int64_t n;
    const double* org;
    int64_t org_ld, org_inc;
    double src[3];
    double* hits;
    int64_t hits_ld;
    double* last_hit;
    int64_t last_hit_ld;
    double* dir_out;
    int64_t dir_out_ld;
    double* det_out;
    int64_t det_out_ld;
    double* opl;
    double* atan_h;
    double* atan_v;
    int64_t sh_begin, sh_end, sv_col;
    double* samp_h;
    double* samp_v;
    int32_t* flags;
    akb_leaf_sink sink;
    const double* pert_h;  // (terms, n_h) / (terms, n_v) OPL perturbation tables or NULL
    const double* pert_v;
    int pert_terms;
    int origin0;  // 1: point source at (+0, +0, +0) and mirror 0 with g != 0, j != 0 (mirror_step kOrigin)
    const double* cp_src;  // staging copy done by workgroup 0 (akb_chain_desc.copy_*)
    double* cp_dst;
    int64_t cp_n;
};

// the launch's staging copy (akb_chain_desc.copy_*), by workgroup 0 ahead of its rays: sixteen
// loads in flight per thread (the source may be host memory across PCIe)
__device__ __forceinline__ void stage_copy(const ChainArgs& a) {
    if (a.cp_n <= 0 || blockIdx.x != 0) return;
    constexpr int kB = 16;
    for (int64_t i0 = threadIdx.x; i0 < a.cp_n; i0 += (int64_t)blockDim.x * kB) {
        double v[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            const int64_t i = i0 + (int64_t)k * blockDim.x;
            v[k] = i < a.cp_n ? __builtin_nontemporal_load(a.cp_src + i) : 0.0;
        }
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            const int64_t i = i0 + (int64_t)k * blockDim.x;
            if (i < a.cp_n) a.cp_dst[i] = v[k];
        }
    }
}

// row / column of flat grid index g without a 64-bit division: q = (t + ((g - t) >> 1)) >> (s - 1)
// with t = mulhi(g, m'), exact for every 32-bit g (Granlund & Montgomery 1994, fig. 4.1)
__device__ __forceinline__ void grid_rc(const ChainArgs& a, int64_t g, uint32_t& iv, uint32_t& ih) {
    const uint32_t g32 = (uint32_t)g;
    uint32_t q;
    if (a.n_h == 1) {
        q = g32;
    } else {
        const uint32_t t = __umulhi(g32, a.div_mul);
        q = (t + ((g32 - t) >> 1)) >> (a.div_shift - 1);
    }
    iv = q;
    ih = g32 - q * a.n_h;  // exact: the grid holds fewer than 2^32 rays
}

// trace flags are raised per wave: the condition's lane mask lands in scalar registers and only a
// wave that holds a flagged ray touches the flag word (no per-lane select / or in the common case)
__device__ __forceinline__ void wave_flag(bool cond, int bit, int& fl) {
    if (__ballot(cond)) fl |= bit;
}

// sqrt_cr of a discriminant with the miss flag !(D > 0). Every lane takes the fast core; only a wave
// holding a lane outside its range (a uniform branch) runs the library sqrt, selects it for those
// lanes and evaluates the miss test - an input inside the range is positive, so a wave without such
// a lane cannot miss, and the common case spends two compares on the range and none on the flag.
__device__ __forceinline__ double sqrt_disc(double D, int bit, int& fl) {
    const bool in = in_fast_range(D);
    double s = sqrt_core(D);
    if (__builtin_expect(__ballot(!in) != 0, 0)) {
        const double sl = sqrt(D);
        s = in ? s : sl;
        wave_flag(!(D > 0.0), bit, fl);
    }
    return s;
}

// norm3_inv with its zero flag in the same form: a squared norm inside the fast range is positive
__device__ __forceinline__ void norm3_inv_flag(double x, double y, double z, double& s, double& inv, int bit,
                                               int& fl) {
    const double v = x * x + y * y + z * z;
    const bool in = in_fast_range(v);
    s = sqrt_core(v);
    inv = rcp_core(s);
    if (__builtin_expect(__ballot(!in) != 0, 0)) {
        const double sl = sqrt(v);
        const double il = 1.0 / sl;
        s = in ? s : sl;
        inv = in ? inv : il;
        wave_flag(s == 0.0, bit, fl);
    }
}

struct Ray {
    double l, m, n;  // direction
    double p, q, r;  // origin / last hit
};

// One mirror of the chain in the reference's numpy association order: mirr_ray_intersection
// (EllipseRaytrace3D.py:23-43), the segment length (AKB_raytrace_20250312.py:2884), norm_vector
// (EllipseRaytrace3D.py:66-70) and reflect_ray (:51-54). A y-free (z-free) mirror skips the terms
// whose coefficients are zero: each is an exact +-0 added to a sum that holds the other terms, the
// gradient's y (z) component is exactly +0 (every term +-0, then + h = +0.0), its square adds +0 to
// the norm, and the reflected y (z) component is m - 2A * (+0) = m: the results are the general
// expression's bits (an exactly-zero partial sum could only change the sign of a zero).
// kUnitIn: the incoming direction is a unit vector (grid rays, or any mirror after the first), so
// the reflected direction's norm skips its range test (norm3_inv_unit).
// kOrigin: the ray leaves the point (+0, +0, +0) (the first mirror of a point-source chain whose
// source is the origin, ChainArgs.origin0): every term of B and C with a factor p, q or r is an
// exact +-0, and a +-0 partial sum plus a non-zero term is that term exactly, so for g != 0 (and
// l > 0, always so for grid rays) B = (g l + h m) + i n and for j != 0 C = j - the host checks both
// conditions. The segment length's x - p is x itself.
// kFlagsOnly: the last mirror of a pass whose only output is the flag word (the fused pass 1): the
// miss and zero-normal tests need the hit and the gradient but nothing after them - the reflected
// direction of a unit ray about a unit normal cannot have a zero norm, so its normalisation (and
// the normal's) are skipped. The ray R is left as it came in.
template <int kKind, bool kOPL, bool kHits, bool kUnitIn, bool kOrigin = false, bool kFlagsOnly = false>
__device__ __forceinline__ void mirror_step(const CMirror& Q, Ray& R, double& opl, int k,
                                            int& fl, double* hits, int64_t hits_ld, int lane) {
    const double l = R.l, m = R.m, n = R.n, p = R.p, q = R.q, r = R.r;
    double A, B, C;
    if (kKind == kKindYFree) {
        A = Q.a * (l * l) + Q.c * (n * n) + Q.e * n * l;
        if (kOrigin) {
            B = Q.g * l + Q.i * n;
            C = Q.j;
        } else {
            B = Q.a2 * p * l + Q.c2 * r * n + Q.e * (p * n + r * l) + Q.g * l + Q.i * n;
            C = Q.a * (p * p) + Q.c * (r * r) + Q.e * p * r + Q.g * p + Q.i * r + Q.j;
        }
    } else if (kKind == kKindZFree) {
        A = Q.a * (l * l) + Q.b * (m * m) + Q.d * m * l;
        if (kOrigin) {
            B = Q.g * l + Q.h * m;
            C = Q.j;
        } else {
            B = Q.a2 * p * l + Q.b2 * q * m + Q.d * (p * m + q * l) + Q.g * l + Q.h * m;
            C = Q.a * (p * p) + Q.b * (q * q) + Q.d * p * q + Q.g * p + Q.h * q + Q.j;
        }
    } else {
        A = Q.a * (l * l) + Q.b * (m * m) + Q.c * (n * n) + Q.d * m * l + Q.e * n * l + Q.f * m * n;
        if (kOrigin) {
            B = Q.g * l + Q.h * m + Q.i * n;
            C = Q.j;
        } else {
            B = Q.a2 * p * l + Q.b2 * q * m + Q.c2 * r * n + Q.d * (p * m + q * l) + Q.e * (p * n + r * l) +
                Q.f * (r * m + q * n) + Q.g * l + Q.h * m + Q.i * n;
            C = Q.a * (p * p) + Q.b * (q * q) + Q.c * (r * r) + Q.d * p * q + Q.e * p * r + Q.f * q * r + Q.g * p +
                Q.h * q + Q.i * r + Q.j;
        }
    }
    const double D = B * B - 4.0 * A * C;
    const double sD = sqrt_disc(D, AKB_FLAG_MISS << (4 * k), fl);
    const double t = div_w(-B + sD * Q.sgn, 2.0 * A);  // (-B - sD) / (2A) for the minus root
    const double x = t * l + p, y = t * m + q, z = t * n + r;
    if (kOPL) {  // opl starts at +0.0: 0 + d is d exactly
        if (kOrigin)
            opl = opl + norm3(x, y, z);
        else
            opl = opl + norm3(x - p, y - q, z - r);
    }
    if (kFlagsOnly) {
        double nx, ny = 0.0, nz = 0.0;
        if (kKind == kKindYFree) {
            nx = Q.a2 * x + Q.e * z + Q.g;
            nz = Q.c2 * z + Q.e * x + Q.i;
        } else if (kKind == kKindZFree) {
            nx = Q.a2 * x + Q.d * y + Q.g;
            ny = Q.b2 * y + Q.d * x + Q.h;
        } else {
            nx = Q.a2 * x + Q.d * y + Q.e * z + Q.g;
            ny = Q.b2 * y + Q.d * x + Q.f * z + Q.h;
            nz = Q.c2 * z + Q.e * x + Q.f * y + Q.i;
        }
        // np.linalg.norm == 0 exactly when the sum of squares is 0
        wave_flag(nx * nx + ny * ny + nz * nz == 0.0, AKB_FLAG_ZERO_NORMAL << (4 * k), fl);
        return;
    }
    // hits: this segment's column 0 of mirror 0's x row (wave-uniform). A compile-time switch: a
    // vector store anywhere in the mirror loop makes the compiler drain every outstanding load
    // before the loop (no separate store counter on gfx9), which would stall the fused kernel's
    // in-flight tilt loads
    if (kHits) {
        double* h = hits + (int64_t)k * 3 * hits_ld;
        h[lane] = x;
        (h + hits_ld)[lane] = y;
        (h + 2 * hits_ld)[lane] = z;
    }
    // unit normal
    double nx, ny = 0.0, nz = 0.0, sn, in;
    const int zbit = AKB_FLAG_ZERO_NORMAL << (4 * k);
    if (kKind == kKindYFree) {
        nx = Q.a2 * x + Q.e * z + Q.g;
        nz = Q.c2 * z + Q.e * x + Q.i;
        norm3_inv_flag(nx, 0.0, nz, sn, in, zbit, fl);
    } else if (kKind == kKindZFree) {
        nx = Q.a2 * x + Q.d * y + Q.g;
        ny = Q.b2 * y + Q.d * x + Q.h;
        norm3_inv_flag(nx, ny, 0.0, sn, in, zbit, fl);
    } else {
        nx = Q.a2 * x + Q.d * y + Q.e * z + Q.g;
        ny = Q.b2 * y + Q.d * x + Q.f * z + Q.h;
        nz = Q.c2 * z + Q.e * x + Q.f * y + Q.i;
        norm3_inv_flag(nx, ny, nz, sn, in, zbit, fl);
    }
    nx = div_pos(nx, sn, in);
    if (kKind != kKindYFree) ny = div_pos(ny, sn, in);
    if (kKind != kKindZFree) nz = div_pos(nz, sn, in);
    // reflection
    double rx, ry, rz;
    if (kKind == kKindYFree) {
        const double A2 = 2.0 * (l * nx + n * nz);
        rx = l - A2 * nx;
        ry = m;
        rz = n - A2 * nz;
    } else if (kKind == kKindZFree) {
        const double A2 = 2.0 * (l * nx + m * ny);
        rx = l - A2 * nx;
        ry = m - A2 * ny;
        rz = n;
    } else {
        const double A2 = 2.0 * (l * nx + m * ny + n * nz);
        rx = l - A2 * nx;
        ry = m - A2 * ny;
        rz = n - A2 * nz;
    }
    double sr, ir;
    if (kUnitIn) {
        bool zero;
        norm3_inv_unit(rx, ry, rz, sr, ir, zero);
        wave_flag(zero, AKB_FLAG_ZERO_REFLECT << (4 * k), fl);
    } else {
        norm3_inv_flag(rx, ry, rz, sr, ir, AKB_FLAG_ZERO_REFLECT << (4 * k), fl);
    }
    R.l = div_pos(rx, sr, ir);
    R.m = div_pos(ry, sr, ir);
    R.n = div_pos(rz, sr, ir);
    R.p = x;
    R.q = y;
    R.r = z;
}

// One ray through the chain: ray i = i0 + t of a segment starting at the wave-uniform i0, t the
// lane's position in it, so every per-ray output row is addressed as a scalar base plus a 32-bit
// lane offset (no per-row 64-bit vector addresses held across the loop). Writes the requested
// per-ray outputs and returns the sink quantities (arctan of the exit slopes and the detector hit)
// in qv.
struct NoHook {
    __device__ __forceinline__ void operator()() const {}
};

// grid position and direction-table entries of flat ray i of a launch
__device__ __forceinline__ void ray_tables(const ChainArgs& a, int64_t i, uint32_t& iv, uint32_t& ih, double& th,
                                           double& tv) {
    grid_rc(a, a.g0 + i * a.g_stride, iv, ih);
    th = ld_off(a.tan_h, ih << 3);  // the tables hold fewer than 2^29 entries (checked on the host)
    tv = ld_off(a.tan_v, iv << 3);
}

// One ray through the chain: ray i = i0 + t of a segment starting at the wave-uniform i0, t the
// lane's position in it, so every per-ray output row is addressed as a scalar base plus a 32-bit
// lane offset (no per-row 64-bit vector addresses held across the loop). Grid rays come with
// their table entries th / tv (iv, ih: grid row and column). Writes the requested per-ray outputs
// and returns the sink quantities (arctan of the exit slopes and the detector hit) in qv.
//
// post(): called after the mirror arithmetic and before any output store. The pipelined kernels
// issue the next segment's loads there: gfx9 counts loads and stores on one in-order counter
// (vmcnt), so loads issued after this segment's stores would make the next segment's first use
// wait for those stores to reach memory; issued before them, they fly during the stores, the leaf
// sums and (for the fused kernels) the next segment's mirror loop.
// kLean: pass 1 of the fused kernel - only the flags leave the ray (the last mirror flags-only; no
// optional output rows, no out-of-line atan call).
// kPointSrc: rays start at the constant source (no origin loads, which would have to be waited
// for - with everything issued before them - ahead of the mirror loop).
// kFixed: pass 2's output set, known at compile time - last hit, exit direction and OPL rows, no
// detector / arctan rows, hits or picks - so none of the optional rows is tested per segment (their
// tests' masks were what overflowed the scalar registers into VGPR lanes).
template <bool kGrid, bool kOPL, bool kNeedQ, bool kHits = false, bool kLean = false, bool kPointSrc = kLean,
          bool kFixed = false, class Post = NoHook>
__device__ __forceinline__ void chain_ray_tab(const ChainArgs& a, int64_t i0, int t, uint32_t iv, uint32_t ih,
                                              double th, double tv, int& fl, double (&qv)[5], Post post = Post()) {
    const int64_t i = i0 + t;
    const int64_t g = a.g0 + i * a.g_stride;
    double* const hits = kHits ? a.hits + i0 : nullptr;
    Ray R;
    if (kGrid) {
        // phai0[:, iv*n_h + ih] = (1, tan(p0h[ih]), tan(p0v[iv])) normalised (ref :2711-2717)
        double s, inv;
        norm3_inv_flag(1.0, th, tv, s, inv, AKB_FLAG_CHAIN_DIR, fl);
        R.l = inv;  // = RN(1/s): also the shared reciprocal
        R.m = div_pos(th, s, inv);
        R.n = div_pos(tv, s, inv);
    } else {
        R.l = a.dir[i * a.dir_inc];
        R.m = a.dir[a.dir_ld + i * a.dir_inc];
        R.n = a.dir[2 * a.dir_ld + i * a.dir_inc];
    }
    if (!kPointSrc && a.org) {
        R.p = a.org[i * a.org_inc];
        R.q = a.org[a.org_ld + i * a.org_inc];
        R.r = a.org[2 * a.org_ld + i * a.org_inc];
    } else {
        R.p = a.src[0];
        R.q = a.src[1];
        R.r = a.src[2];
    }
    double opl = 0.0;
    // the first mirror from the origin (a point source at +0, ChainArgs.origin0) and the last
    // mirror of a flags-only pass take their reduced forms (mirror_step's kOrigin / kFlagsOnly)
    int k0 = 0;
    const int kend = kLean ? a.K - 1 : a.K;
    if (kGrid && a.origin0) {  // wave-uniform (grid rays: l > 0)
        if (kLean && a.K == 1) {
            if (a.kind[0] == kKindYFree)
                mirror_step<kKindYFree, kOPL, kHits, kGrid, true, true>(a.q[0], R, opl, 0, fl, hits, a.hits_ld, t);
            else if (a.kind[0] == kKindZFree)
                mirror_step<kKindZFree, kOPL, kHits, kGrid, true, true>(a.q[0], R, opl, 0, fl, hits, a.hits_ld, t);
            else
                mirror_step<kKindGeneral, kOPL, kHits, kGrid, true, true>(a.q[0], R, opl, 0, fl, hits, a.hits_ld, t);
            k0 = 1;
        } else {
            if (a.kind[0] == kKindYFree)
                mirror_step<kKindYFree, kOPL, kHits, kGrid, true>(a.q[0], R, opl, 0, fl, hits, a.hits_ld, t);
            else if (a.kind[0] == kKindZFree)
                mirror_step<kKindZFree, kOPL, kHits, kGrid, true>(a.q[0], R, opl, 0, fl, hits, a.hits_ld, t);
            else
                mirror_step<kKindGeneral, kOPL, kHits, kGrid, true>(a.q[0], R, opl, 0, fl, hits, a.hits_ld, t);
            k0 = 1;
        }
    }
    // not unrolled: each iteration reads its mirror's coefficients from the kernel argument segment
    // with scalar loads (wave-uniform), keeping VGPR pressure and code size low (a fully unrolled
    // 4-mirror AKB kernel measured 12 % slower on MI355X)
#pragma unroll 1
    for (int k = k0; k < kend; ++k) {
        if (a.kind[k] == kKindYFree)  // wave-uniform branch
            mirror_step<kKindYFree, kOPL, kHits, kGrid>(a.q[k], R, opl, k, fl, hits, a.hits_ld, t);
        else if (a.kind[k] == kKindZFree)
            mirror_step<kKindZFree, kOPL, kHits, kGrid>(a.q[k], R, opl, k, fl, hits, a.hits_ld, t);
        else
            mirror_step<kKindGeneral, kOPL, kHits, kGrid>(a.q[k], R, opl, k, fl, hits, a.hits_ld, t);
    }
    if (kLean && kend >= k0) {  // the last mirror: its flags only
        const int k = kend;
        if (a.kind[k] == kKindYFree)
            mirror_step<kKindYFree, kOPL, kHits, kGrid, false, true>(a.q[k], R, opl, k, fl, hits, a.hits_ld, t);
        else if (a.kind[k] == kKindZFree)
            mirror_step<kKindZFree, kOPL, kHits, kGrid, false, true>(a.q[k], R, opl, k, fl, hits, a.hits_ld, t);
        else
            mirror_step<kKindGeneral, kOPL, kHits, kGrid, false, true>(a.q[k], R, opl, k, fl, hits, a.hits_ld, t);
    }
    const double l = R.l, m = R.m, nn = R.n, p = R.p, q = R.q, r = R.r;
    if (kOPL && kGrid && a.pert_h) {  // figure-error perturbation of the path (BASELINE config 5)
        double d = 0.0;
        for (int k = 0; k < a.pert_terms; ++k)
            d = __builtin_fma(a.pert_v[(int64_t)k * a.n_v + iv], a.pert_h[(int64_t)k * a.n_h + ih], d);
        opl = opl + d;
    }
    post();
    const uint32_t off = (uint32_t)t << 3;
    if (kOPL && (kFixed || a.opl)) st_off(a.opl + i0, off, opl);
    if (!kLean && (kFixed || a.last_hit)) {
        double* o = a.last_hit + i0;
        st_off(o, off, p);
        st_off(o + a.last_hit_ld, off, q);
        st_off(o + 2 * a.last_hit_ld, off, r);
    }
    if (!kLean && (kFixed || a.dir_out)) {
        double* o = a.dir_out + i0;
        st_off(o, off, l);
        st_off(o + a.dir_out_ld, off, m);
        st_off(o + 2 * a.dir_out_ld, off, nn);
    }
    if (kNeedQ || (!kLean && !kFixed && a.det_out)) {
        double x, y, z;
        plane_hit(a.det[0], a.det[1], a.det[2], a.det[3], l, m, nn, p, q, r, x, y, z);
        if (!kLean && !kFixed && a.det_out) {
            double* o = a.det_out + i0;
            o[t] = x;
            (o + a.det_out_ld)[t] = y;
            (o + 2 * a.det_out_ld)[t] = z;
        }
        qv[2] = x;
        qv[3] = y;
        qv[4] = z;
    }
    if (kNeedQ || (!kLean && !kFixed && (a.atan_h || a.atan_v))) {
        const double il = div_w(1.0, l);
        qv[0] = atan_slope(div_shared(m, l, il));
        qv[1] = atan_slope(div_shared(nn, l, il));
        if (!kFixed && a.atan_h) (a.atan_h + i0)[t] = qv[0];
        if (!kFixed && a.atan_v) (a.atan_v + i0)[t] = qv[1];
    }
    if (kFixed) return;
    // equal-angle resample samples: the slope ratios only; the host applies np.arctan so the
    // resampled angle tables match the reference bit for bit (glibc atan, ref :2858-2859)
    if (a.samp_h && g >= a.sh_begin && g < a.sh_end) a.samp_h[g - a.sh_begin] = m / l;
    if (a.samp_v && kGrid && ih == a.sv_col) a.samp_v[iv] = nn / l;
}

// the same, loading its own table entries (the unpipelined kernels)
template <bool kGrid, bool kOPL, bool kNeedQ, bool kHits = false, bool kLean = false, bool kPointSrc = kLean,
          bool kFixed = false>
__device__ __forceinline__ void chain_ray(const ChainArgs& a, int64_t i0, int t, int& fl, double (&qv)[5]) {
    uint32_t iv = 0, ih = 0;
    double th = 0.0, tv = 0.0;
    if (kGrid) ray_tables(a, i0 + t, iv, ih, th, tv);
    chain_ray_tab<kGrid, kOPL, kNeedQ, kHits, kLean, kPointSrc, kFixed>(a, i0, t, iv, ih, th, tv, fl, qv);
}

template <bool kGrid, bool kOPL, int kWaves, bool kHits = false, bool kPointSrc = false>
__global__ void __launch_bounds__(kBlock, kWaves) k_chain(ChainArgs a) {
    stage_copy(a);
    int fl = 0;
    double qv[5];
    const int t = threadIdx.x;
    for (int64_t i0 = blockIdx.x * (int64_t)kBlock; i0 < a.n; i0 += (int64_t)gridDim.x * kBlock)
        if (i0 + t < a.n) chain_ray<kGrid, kOPL, false, kHits, false, kPointSrc>(a, i0, t, fl, qv);
    if (fl) atomicOr(a.flags, fl);
}

// the same, walking 256-ray segments and feeding the fused np.nanmean(arctan) / np.mean(det)
// leaf sums (the tilt means, ref :3583-3591) instead of writing those five rows to HBM
// kPointSrc: grid rays from the point source (no origin loads)
// kFixed: pass 2 of RayWave (chain_ray_tab's fixed output set)
template <bool kGrid, bool kOPL, int kWaves, bool kPointSrc = false, bool kFixed = false>
__global__ void __launch_bounds__(kBlock, kWaves) k_chain_sink(ChainArgs a) {
    stage_copy(a);
    __shared__ LeafLds<5> L;
    int fl = 0;
    const int t = threadIdx.x;
    const int64_t nseg = (a.n + kLeafSeg - 1) / kLeafSeg;
    for (int64_t seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
        const bool valid = seg * kLeafSeg + t < a.n;
        double qv[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
        if (valid) chain_ray<kGrid, kOPL, true, false, false, kPointSrc, kFixed>(a, seg * kLeafSeg, t, fl, qv);
        leaf_sink_segment<5>(a.sink, L, seg * kLeafSeg, qv, valid);
    }
    if (fl) atomicOr(a.flags, fl);
}

// S independent grid systems in one launch: auto_focus_NA and calc_FoC trace many small systems
// that differ in their mirrors, launch tables or source (ref AKB_raytrace_20250312.py:12776-12786,
// :13780-13784). blockIdx.y picks the system; its kernel arguments sit in device memory at a
// wave-uniform address, so every field is a scalar load, as from the argument segment.
template <bool kOPL, bool kHits>
__global__ void __launch_bounds__(kBlock) k_chain_batch(const ChainArgs* __restrict__ A) {
    const ChainArgs& a = A[blockIdx.y];
    int fl = 0;
    double qv[5];
    const int t = threadIdx.x;
    for (int64_t i0 = blockIdx.x * (int64_t)kBlock; i0 < a.n; i0 += (int64_t)gridDim.x * kBlock)
        if (i0 + t < a.n) chain_ray<true, kOPL, false, kHits, false, false>(a, i0, t, fl, qv);
    if (fl) atomicOr(a.flags, fl);
}

// ----------------------------------------------------------------------------------------------
// tilt correction + detectors + OPL (ref AKB_raytrace_20250312.py:3583-3601, :3611-3633)
// ----------------------------------------------------------------------------------------------

// Parameter block of the tilt (ref :3583-3591 and rotate_vectors :917-927), formed on the device
// from the pass-2 sums so no host round trip sits between pass 2 and the tilt:
//   theta_y = -nanmean(arctan(Rz/Rx)), theta_z = nanmean(arctan(Ry/Rx)), focus = mean(det)
//   Ry, Rz = rotation_matrices(-theta_y, -theta_z) with correctly rounded cos / sin
// It also zeroes the words the next step accumulates into (pupil extent keys, trace flags that
// were already copied out in stream order).
constexpr int kTiltTheta = 0, kTiltRy = 2, kTiltRz = 11, kTiltFocus = 20, kTiltSaved = 23;

// the parameter block from the five sums / counts, by one 64-lane wave (the whole of k_tilt_params,
// and the last step of k_finish_params)
__device__ __forceinline__ void tilt_params_wave(const double* s5, const int64_t* c5, double* P,
                                                 unsigned long long* keys, int32_t* clear, int nclear, int lane);

__global__ void k_tilt_params(const double* __restrict__ s5, const int64_t* __restrict__ c5, double* __restrict__ P,
                              unsigned long long* keys, int32_t* clear, int nclear) {
    tilt_params_wave(s5, c5, P, keys, clear, nclear, threadIdx.x);
}

__device__ __forceinline__ void tilt_params_wave(const double* s5, const int64_t* c5, double* P,
                                                 unsigned long long* keys, int32_t* clear, int nclear, int lane) {
    // np.nanmean / np.mean: sum / count, an IEEE division (0 / 0 -> NaN as numpy's)
    const double mh = s5[0] / (double)c5[0];
    const double mv = s5[1] / (double)c5[1];
    const double theta_y = -mv, theta_z = mh;
    // lanes 0..3: sin(-theta_y), cos(-theta_y), sin(-theta_z), cos(-theta_z) side by side
    double v = 0.0;
    if (lane < 4) v = akb_sc::sin_cos_cr(lane < 2 ? -theta_y : -theta_z, lane & 1);
    const double sy = __shfl(v, 0), cy = __shfl(v, 1), sz = __shfl(v, 2), cz = __shfl(v, 3);
    if (lane == 0) {
        P[kTiltTheta] = theta_y;
        P[kTiltTheta + 1] = theta_z;
        const double ry[9] = {cy, 0.0, sy, 0.0, 1.0, 0.0, -sy, 0.0, cy};
        const double rz[9] = {cz, -sz, 0.0, sz, cz, 0.0, 0.0, 0.0, 1.0};
        for (int k = 0; k < 9; ++k) {
            P[kTiltRy + k] = ry[k];
            P[kTiltRz + k] = rz[k];
        }
    }
    if (lane >= 4 && lane < 7) P[kTiltFocus + lane - 4] = s5[2 + lane - 4] / (double)c5[2 + lane - 4];
    if (keys && lane < 4) keys[lane] = 0ULL;
    // the first (up to 4) words are kept in the block before they are cleared, so the host can
    // read them from there whenever it likes (RayWave's trace flag words)
    if (lane < 4) ((int32_t*)(P + kTiltSaved))[lane] = lane < nclear ? clear[lane] : 0;
    __syncthreads();
    for (int i = lane; i < nclear; i += 64) clear[i] = 0;
}

// The pass-2 sink's finish and the tilt parameters in two launches instead of three
// (akb_leaf_finish_f64's k_leaf_chunks + k_pw_final, then k_tilt_params): on the critical path of a
// ray_wave run every kernel boundary costs ~10 us.
// k_fin_buffers (256 threads): block (b, q) forms the sums of buffers b*kFinBPB .. +kFinBPB-1 of
// quantity q from their 64 leaf sums each (numpy's tree over a buffer's leaves; a wave per buffer
// group, all loads in flight together); the last block of each quantity instead stages the short
// last buffer in LDS (NaN -> 0 for the nanmean rows) and forms its pairwise sum and count.
// k_fin_params (one workgroup, wave q for quantity q): the buffer sums staged in LDS and added left
// to right, the short buffer last - numpy's order - then wave 0 forms the parameter block. No
// cross-workgroup hand-off inside a kernel, so no device-scope fences.
constexpr int kFinBPB = 32;      // buffers per k_fin_buffers block (8 per wave)
constexpr int kFinTile = 512;    // buffer sums staged per LDS round and wave (20 KB of LDS: the
                                 // kernel then fits beside the trace passes instead of waiting for a CU to drain)

__global__ void __launch_bounds__(256) k_fin_buffers(akb_leaf_sink S, int64_t nfull, double* __restrict__ part,
                                                     long long* __restrict__ part_cnt) {
    AKB_CHAIN_PRIORITY();
    extern __shared__ double tl[];  // the short buffer (its length in doubles)
    __shared__ PwTree T;
    const int q = blockIdx.y;
    const int64_t blk = blockIdx.x;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t nb = (nfull + kFinBPB - 1) / kFinBPB;
    double* const tsum = part + (int64_t)S.nq * nfull;
    long long* const tcnt = part_cnt + (int64_t)S.nq * nfull;
    if (blk < nb) {
        constexpr int kPer = kFinBPB / 4;
        const int64_t nleaves = nfull * (kNpBuf / 128);
        double v[kPer];
        int k[kPer];
#pragma unroll
        for (int b = 0; b < kPer; ++b) {
            const int64_t c = blk * kFinBPB + w * kPer + b;
            const int64_t li = (int64_t)q * nleaves + c * 64 + lane;
            v[b] = c < nfull ? S.leaf_sum[li] : 0.0;
            k[b] = c < nfull ? S.leaf_cnt[li] : 0;
        }
#pragma unroll
        for (int b = 0; b < kPer; ++b) {
            double x = v[b];
            x = x + __shfl_xor(x, 1);
            x = x + __shfl_xor(x, 2);
            x = x + __shfl_xor(x, 4);
            x = x + __shfl_xor(x, 8);
            x = x + __shfl_xor(x, 16);
            x = x + __shfl_xor(x, 32);
            long long kk = k[b];
            for (int off = 32; off > 0; off >>= 1) kk += __shfl_down(kk, off);
            const int64_t c = blk * kFinBPB + w * kPer + b;
            if (lane == 0 && c < nfull) {
                part[(int64_t)q * nfull + c] = x;
                part_cnt[(int64_t)q * nfull + c] = kk;
            }
        }
        return;
    }
    // the short last buffer
    const int tail = (int)(S.n - nfull * kNpBuf);
    const bool nan0 = (S.nan_mask >> (q < 31 ? q : 31)) & 1;
    const double* a = S.tail + (int64_t)q * kNpBuf;
    long long cnt = 0;
    for (int i = threadIdx.x; i < tail; i += 256) tl[i] = nan_zero(a[i], nan0, cnt);
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off);
    __shared__ long long wc[4];
    if (lane == 0) wc[w] = cnt;
    __syncthreads();
    if (w == 0) {
        const double v = tail > 0 ? pw_tree_wave(T, tl, tail) : 0.0;
        if (lane == 0) {
            tsum[q] = v;
            tcnt[q] = wc[0] + wc[1] + wc[2] + wc[3];
        }
    }
}

__global__ void __launch_bounds__(320) k_fin_params(akb_leaf_sink S, int64_t nfull, const double* __restrict__ part,
                                                    const long long* __restrict__ part_cnt, double* __restrict__ sum5,
                                                    int64_t* __restrict__ cnt5, double* __restrict__ P,
                                                    unsigned long long* keys, int32_t* clear, int nclear) {
    AKB_CHAIN_PRIORITY();
    __shared__ double tile[5][kFinTile];
    __shared__ double s5[8];
    __shared__ int64_t c5[8];
    const int q = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tail = (int)(S.n - nfull * kNpBuf);
    long long cnt = 0;
    double acc = 0.0;
    const double* pq = part + (int64_t)q * nfull;
    const long long* cq = part_cnt + (int64_t)q * nfull;
    for (int64_t base = 0; base < nfull; base += kFinTile) {
        const int m = (int)(nfull - base < kFinTile ? nfull - base : kFinTile);
        constexpr int kB = kFinTile / 64;
        double vb[kB];
#pragma unroll
        for (int r = 0; r < kB; ++r) {
            const int i = lane + 64 * r;
            vb[r] = i < m ? pq[base + i] : 0.0;
            cnt += i < m ? cq[base + i] : 0;
        }
#pragma unroll
        for (int r = 0; r < kB; ++r) {
            const int i = lane + 64 * r;
            if (i < m) tile[q][i] = vb[r];
        }
        wave_sync();
        if (lane == 0) {  // 16 LDS reads in flight ahead of 16 dependent adds
            int i = 0;
            if (base == 0) {
                acc = tile[q][0];
                i = 1;
            }
            double u[16];
            for (; i + 16 <= m; i += 16) {
#pragma unroll
                for (int r = 0; r < 16; ++r) u[r] = tile[q][i + r];
#pragma unroll
                for (int r = 0; r < 16; ++r) acc = acc + u[r];
            }
            for (; i < m; ++i) acc = acc + tile[q][i];
        }
        wave_sync();
    }
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off);
    if (lane == 0) {
        const double* tsum = part + (int64_t)S.nq * nfull;
        const long long* tcnt = part_cnt + (int64_t)S.nq * nfull;
        const double sv = tail > 0 ? (nfull > 0 ? acc + tsum[q] : tsum[q]) : acc;
        const long long cv = cnt + (tail > 0 ? tcnt[q] : 0);
        s5[q] = sv;
        c5[q] = cv;
        sum5[q] = sv;
        cnt5[q] = cv;
    }
    __syncthreads();
    if (q == 0) tilt_params_wave(s5, c5, P, keys, clear, nclear, lane);
}

__device__ __forceinline__ void tilt_ray(const TiltArgs& a, int64_t i, const TiltIn& t, double (&qv)[5]) {
    double ax, ay, az;
    double l, m, n;
    matvec(a.Rz, t.d[0], t.d[1], t.d[2], ax, ay, az);
    matvec(a.Ry, ax, ay, az, l, m, n);
    double p, q, r;
    matvec(a.Rz, t.p[0] - a.c[0], t.p[1] - a.c[1], t.p[2] - a.c[2], ax, ay, az);
    matvec(a.Ry, ax, ay, az, p, q, r);
    p = p + a.c[0];
    q = q + a.c[1];
    r = r + a.c[2];
    if (a.dir_rot) {
        a.dir_rot[i] = l;
        a.dir_rot[a.ld + i] = m;
        a.dir_rot[2 * a.ld + i] = n;
    }
    if (a.pt_rot) {
        a.pt_rot[i] = p;
        a.pt_rot[a.ld + i] = q;
        a.pt_rot[2 * a.ld + i] = r;
    }
    const double o = t.o;
    double x, y, z;
    plane_hit(a.d1[0], a.d1[1], a.d1[2], a.d1[3], l, m, n, p, q, r, x, y, z);
    if (a.det1) {
        a.det1[i] = x;
        a.det1[a.ld + i] = y;
        a.det1[2 * a.ld + i] = z;
    }
    qv[0] = x;
    qv[1] = y;
    qv[2] = z;
    qv[3] = o + norm3(x - p, y - q, z - r);
    if (a.total1) a.total1[i] = qv[3];
    plane_hit(a.d2[0], a.d2[1], a.d2[2], a.d2[3], l, m, n, p, q, r, x, y, z);
    if (a.det2) {
        a.det2[i] = x;
        a.det2[a.ld + i] = y;
        a.det2[2 * a.ld + i] = z;
    }
    qv[4] = o + norm3(x - p, y - q, z - r);
    if (a.total2) a.total2[i] = qv[4];
}

// tilt_ray's arithmetic without its stores (the fused kernel computes before issuing the next
// segment's loads and stores after): detector-2 hit and total OPL 2 in d2 / t2, the sink
// quantities (detector-1 hit, total OPL 1, total OPL 2) in qv
__device__ __forceinline__ void tilt_compute(const TiltArgs& a, const TiltIn& t, double (&d2)[3], double (&qv)[5]) {
    double ax, ay, az;
    double l, m, n;
    matvec(a.Rz, t.d[0], t.d[1], t.d[2], ax, ay, az);
    matvec(a.Ry, ax, ay, az, l, m, n);
    double p, q, r;
    matvec(a.Rz, t.p[0] - a.c[0], t.p[1] - a.c[1], t.p[2] - a.c[2], ax, ay, az);
    matvec(a.Ry, ax, ay, az, p, q, r);
    p = p + a.c[0];
    q = q + a.c[1];
    r = r + a.c[2];
    double x, y, z;
    plane_hit(a.d1[0], a.d1[1], a.d1[2], a.d1[3], l, m, n, p, q, r, x, y, z);
    qv[0] = x;
    qv[1] = y;
    qv[2] = z;
    qv[3] = t.o + norm3(x - p, y - q, z - r);
    plane_hit(a.d2[0], a.d2[1], a.d2[2], a.d2[3], l, m, n, p, q, r, x, y, z);
    d2[0] = x;
    d2[1] = y;
    d2[2] = z;
    qv[4] = t.o + norm3(x - p, y - q, z - r);
}

__device__ __forceinline__ void tilt_store(const TiltArgs& a, int64_t i0, int t, const double (&d2)[3],
                                           const double (&qv)[5]) {
    if (a.det1) {
        double* o = a.det1 + i0;
        o[t] = qv[0];
        (o + a.ld)[t] = qv[1];
        (o + 2 * a.ld)[t] = qv[2];
    }
    if (a.total1) (a.total1 + i0)[t] = qv[3];
    if (a.det2) {
        double* o = a.det2 + i0;
        o[t] = d2[0];
        (o + a.ld)[t] = d2[1];
        (o + 2 * a.ld)[t] = d2[2];
    }
    if (a.total2) (a.total2 + i0)[t] = qv[4];
}

// the rotation and centre from the device parameter block (uniform scalar loads)
__device__ __forceinline__ void tilt_load_params(TiltArgs& a) {
    if (!a.params) return;
    const double* P = a.params;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        a.Ry.m[k] = P[kTiltRy + k];
        a.Rz.m[k] = P[kTiltRz + k];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) a.c[k] = P[kTiltFocus + k];
}

__global__ void __launch_bounds__(kBlock) k_tilt_opd(TiltArgs a) {
    tilt_load_params(a);
    double qv[5];
    TiltIn t;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < a.n;
         i += (int64_t)gridDim.x * blockDim.x) {
        tilt_load(a, i, t);
        tilt_ray(a, i, t, qv);
    }
}

// the next segment's inputs are loaded before this segment's arithmetic and leaf sums, so each
// wave keeps its loads in flight across the sink's barriers
__global__ void __launch_bounds__(kBlock) k_tilt_opd_sink(TiltArgs a) {
    tilt_load_params(a);
    __shared__ LeafLds<5> L;
    const int64_t nseg = (a.n + kLeafSeg - 1) / kLeafSeg;
    int64_t seg = blockIdx.x;
    TiltIn cur{}, nxt{};
    {
        const int64_t i = seg * kLeafSeg + threadIdx.x;
        if (seg < nseg && i < a.n) tilt_load(a, i, cur);
    }
    for (; seg < nseg; seg += gridDim.x) {
        const int64_t i = seg * kLeafSeg + threadIdx.x;
        const bool valid = i < a.n;
        const int64_t j = (seg + gridDim.x) * kLeafSeg + threadIdx.x;
        if (seg + gridDim.x < nseg && j < a.n) tilt_load(a, j, nxt);
        double qv[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
        if (valid) tilt_ray(a, i, cur, qv);
        leaf_sink_segment<5>(a.sink, L, seg * kLeafSeg, qv, valid);
        cur = nxt;
    }
}

// order-preserving uint64 key of a double (larger double -> larger key); 0 is below every key
__device__ __forceinline__ unsigned long long order_key(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ULL);
}
__device__ __forceinline__ double key_value(unsigned long long k) {
    const unsigned long long b = (k >> 63) ? (k & 0x7fffffffffffffffULL) : ~k;
    return __longlong_as_double((long long)b);
}

struct OpdArgs {
    const double* t1;
    const double* t2;
    const double* det2;
    int64_t ld, n;
    const double* sum5;
    const int64_t* cnt5;
    double* e1;
    double* e2;
    double* sph;
    double* wave;
    unsigned long long* ext;
};

// the fused kernel's OPD rows (akb_chain_tilt_opd_f64; ld / n are the tilt's)
struct OpdRows {
    const double* t2;
    const double* det2;
    double* e2;
    double* wave;
    unsigned long long* ext;
    const double* sum5;
    const int64_t* cnt5;
};

// one ray's OPD inputs (ref :3633, :3675-3677): total2 and the detector-2 point
struct OpdIn {
    double t2, x, y, z;
};
__device__ __forceinline__ void opd_load(const OpdRows& o, int64_t ld, int64_t i0, uint32_t off, OpdIn& v) {
    const double* d = o.det2 + i0;
    v.t2 = ld_off(o.t2 + i0, off);
    v.x = ld_off(d, off);
    v.y = ld_off(d + ld, off);
    v.z = ld_off(d + 2 * ld, off);
}

// the workgroup's four extents (max y, -y, z, -z) folded into the device keys (thread-uniform
// call: every thread of the workgroup reaches it)
__device__ __forceinline__ void extents_commit(double (&e)[4], unsigned long long* ext) {
    __shared__ double wext[kBlock / 64][4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        for (int off = 32; off > 0; off >>= 1) e[k] = fmax(e[k], __shfl_down(e[k], off));
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 4; ++k) wext[threadIdx.x >> 6][k] = e[k];
    __syncthreads();
    if (threadIdx.x < 4) {
        double v = wext[0][threadIdx.x];
        for (int w = 1; w < kBlock / 64; ++w) v = fmax(v, wext[w][threadIdx.x]);
        const unsigned long long k = order_key(v);
        // most workgroups hold no new extreme: skip their atomic (the max stays exact)
        if (k > __hip_atomic_load(ext + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            atomicMax(ext + threadIdx.x, k);
    }
}

// Pass 1 of one run fused with the tilt of the run before it (RayWave.launch_front(fuse=...)):
// both walk the same shard in 256-ray segments. Each segment's tilt inputs (56 B per ray, written
// by the previous run's pass 2) are loaded right after the ray's grid-table loads and arrive
// while the FP64-bound mirror chain runs, so the tilt's HBM traffic hides behind pass 1's
// arithmetic instead of competing with it for wave slots as a second kernel would.
//
// kOPD: the same kernel also forms the OPD maps of the run before that one (o: its tilt outputs
// and tilt sums, RayWave.launch_front(fuse_opd=...)), 48 B per ray more behind the same chain:
// Wave2 = DistError2 - Sph, and the detector-2 extents for the pupil pitch.
template <int kWaves, bool kOPD>
__global__ void __launch_bounds__(kBlock, kWaves) k_chain_tilt(ChainArgs a, TiltArgs b, OpdRows o) {
    stage_copy(a);
    tilt_load_params(b);
    // the OPD's means and each thread's running extents live in LDS, and its inputs are loaded
    // for the current segment only (issued ahead of the tilt arithmetic, which hides part of their
    // latency): nothing of the OPD is live across the mirror loop
    __shared__ double om[kOPD ? 4 : 1];
    __shared__ double oe[kOPD ? 4 : 1][kOPD ? kBlock : 1];
    if constexpr (kOPD) {
        if (threadIdx.x < 4) {  // np.nanmean results, as k_opd forms them: f0, f1, f2, mean2
            const int q = threadIdx.x == 3 ? 4 : threadIdx.x;
            om[threadIdx.x] = o.sum5[q] / (double)o.cnt5[q];
        }
        for (int k = 0; k < 4; ++k) oe[k][threadIdx.x] = -INFINITY;
        __syncthreads();
    }
    __shared__ LeafLds<5> L;
    int fl = 0;
    double qv[5];
    const int t = threadIdx.x;
    const int64_t nseg = (a.n + kLeafSeg - 1) / kLeafSeg;
    int64_t seg = blockIdx.x;
    // software pipeline: segment s's table entries and tilt inputs were loaded during segment
    // s - gridDim's stores, leaf sums and mirror loop
    uint32_t iv = 0, ih = 0;
    double th = 0.0, tv = 0.0;
    TiltIn in;
    if (seg < nseg && seg * kLeafSeg + t < a.n) {
        ray_tables(a, seg * kLeafSeg + t, iv, ih, th, tv);
        tilt_load_seg(b, seg * kLeafSeg, (uint32_t)t << 3, in);
    }
    for (; seg < nseg; seg += gridDim.x) {
        // the thread index made opaque per segment: addresses derived from it are formed where
        // they are used instead of being hoisted out of the loop and kept live (or spilled, and
        // reloaded behind the prefetch loads) across the mirror chain
        int t = threadIdx.x;
        asm volatile("" : "+v"(t));
        const int64_t i0 = seg * kLeafSeg;
        const bool valid = i0 + t < a.n;
        const int64_t n0 = (seg + gridDim.x) * kLeafSeg;  // the next segment (wave-uniform)
        const int64_t nxt = n0 + t;
        const uint32_t off = (uint32_t)t << 3;
        double d2[3], tq[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
        if (valid)
            chain_ray_tab<true, false, false, false, true, true>(a, i0, t, iv, ih, th, tv, fl, qv, [&] {
                OpdIn oin;
                if constexpr (kOPD) opd_load(o, b.ld, i0, off, oin);
                tilt_compute(b, in, d2, tq);
                if constexpr (kOPD) {  // k_opd's arithmetic, in its order
                    const double oe2 = (oin.t2 - om[3]) * 1e9;
                    st_off(o.e2 + i0, off, oe2);
                    st_off(o.wave + i0, off, oe2 - norm3(oin.x - om[0], oin.y - om[1], oin.z - om[2]) * 1e9);
                    oe[0][t] = fmax(oe[0][t], oin.y);
                    oe[1][t] = fmax(oe[1][t], -oin.y);
                    oe[2][t] = fmax(oe[2][t], oin.z);
                    oe[3][t] = fmax(oe[3][t], -oin.z);
                }
                if (nxt < a.n) {
                    ray_tables(a, nxt, iv, ih, th, tv);
                    tilt_load_seg(b, n0, off, in);
                }
            });
        if (valid) {  // detector-2 rows only (detector 1 and the rotated rays are the full mode's)
            double* r = b.det2 + i0;
            st_off(r, off, d2[0]);
            st_off(r + b.ld, off, d2[1]);
            st_off(r + 2 * b.ld, off, d2[2]);
            st_off(b.total2 + i0, off, tq[4]);
        }
        leaf_sink_segment<5>(b.sink, L, i0, tq, valid, t);
    }
    if (fl) atomicOr(a.flags, fl);
    if constexpr (kOPD) {
        double e[4] = {oe[0][t], oe[1][t], oe[2][t], oe[3][t]};
        extents_commit(e, o.ext);
    }
}

// ----------------------------------------------------------------------------------------------
// OPD maps + pupil footprint (ref :3626, :3633, :3675-3677)
// ----------------------------------------------------------------------------------------------

__global__ void __launch_bounds__(kBlock) k_opd(OpdArgs a) {
    // np.nanmean results: sum / count in float64 (the reference's true_divide)
    const double f0 = a.sum5[0] / (double)a.cnt5[0];
    const double f1 = a.sum5[1] / (double)a.cnt5[1];
    const double f2 = a.sum5[2] / (double)a.cnt5[2];
    const double mean1 = a.sum5[3] / (double)a.cnt5[3];
    const double mean2 = a.sum5[4] / (double)a.cnt5[4];
    double e[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < a.n;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (a.e1) a.e1[i] = (a.t1[i] - mean1) * 1e9;
        const double e2 = (a.t2[i] - mean2) * 1e9;
        if (a.e2) a.e2[i] = e2;
        const double y = a.det2[a.ld + i], z = a.det2[2 * a.ld + i];
        if (a.sph || a.wave) {
            const double s = norm3(a.det2[i] - f0, y - f1, z - f2) * 1e9;
            if (a.sph) a.sph[i] = s;
            if (a.wave) a.wave[i] = e2 - s;
        }
        if (a.ext) {  // fmax ignores NaN
            e[0] = fmax(e[0], y);
            e[1] = fmax(e[1], -y);
            e[2] = fmax(e[2], z);
            e[3] = fmax(e[3], -z);
        }
    }
    if (a.ext) extents_commit(e, a.ext);
}

__global__ void __launch_bounds__(kBlock) k_pupil(const double* wave, int64_t ray0, int64_t nrays, int64_t n,
                                                  int size, const unsigned long long* ext, double* opd,
                                                  double* pitch) {
    const int64_t total = (int64_t)size * size;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int ky = (int)(k / size), kx = (int)(k - (int64_t)ky * size);
        const int64_t iv = ((int64_t)ky * (n - 1)) / (size - 1);
        const int64_t ih = ((int64_t)kx * (n - 1)) / (size - 1);
        double v = 0.0;
        const int64_t g = iv * n + ih;
        if (g >= ray0 && g < ray0 + nrays) v = wave[g - ray0] * 1e-9;
        opd[k] = v;
    }
    if (pitch && blockIdx.x == 0 && threadIdx.x == 0) {
        pitch[0] = (key_value(ext[0]) + key_value(ext[1])) / (double)(size - 1);
        pitch[1] = (key_value(ext[2]) + key_value(ext[3])) / (double)(size - 1);
    }
}

}  // namespace akb

// ==============================================================================================
// C ABI
// ==============================================================================================

using namespace akb;

static inline V3In v3in(const double* p, int64_t ld, int64_t inc) { return V3In{p, ld, inc}; }

// the chain kernels at 4 waves per SIMD (the register allocator's floor; pass 2's fixed-output
// sink: 89 VGPRs and no scratch; 6 waves spilled 8 VGPRs and was no faster, 8 spilled 160 B and
// was slower), workgroups capped at 8192 (each walks 256-ray segments grid-stride; measured best
// for both passes); the OPD kernel at 2048 (its extent atomics grow with the grid)
constexpr int kChainWaves = 4;
constexpr int64_t kChainGridCap = 256 * 32;
constexpr int64_t kOpdGridCap = 2048;

template <bool kGrid, bool kOPL, bool kSink>
static void launch_chain(int w, unsigned g, hipStream_t s, const ChainArgs& a) {
    if (!kSink && a.hits) {  // per-mirror hit rows (the stage-equivalent outputs): one variant
        k_chain<kGrid, kOPL, 4, true><<<g, kBlock, 0, s>>>(a);
        return;
    }
    // rays from the point source: the variant without origin loads (grid rays only)
    const bool point = kGrid && a.org == nullptr;
    // RayWave's pass 2: exactly the last hit, exit direction and OPL rows
    const bool fixed = kGrid && kOPL && point && a.last_hit && a.dir_out && a.opl && !a.det_out && !a.atan_h &&
                       !a.atan_v && !a.samp_h && !a.samp_v && !a.hits;
    if (kSink && fixed) {
        k_chain_sink<kGrid, kOPL, kChainWaves, kGrid, kGrid && kOPL><<<g, kBlock, 0, s>>>(a);
        return;
    }
    (void)w;
    if (kSink && point)
        k_chain_sink<kGrid, kOPL, kChainWaves, kGrid><<<g, kBlock, 0, s>>>(a);
    else if (kSink)
        k_chain_sink<kGrid, kOPL, kChainWaves, false><<<g, kBlock, 0, s>>>(a);
    else if (point)
        k_chain<kGrid, kOPL, kChainWaves, false, kGrid><<<g, kBlock, 0, s>>>(a);
    else
        k_chain<kGrid, kOPL, kChainWaves, false, false><<<g, kBlock, 0, s>>>(a);
}

extern "C" {

const char* akb_last_error(void) { return g_last_error.c_str(); }
int akb_abi_version(void) { return AKB_ABI_VERSION; }
#ifndef AKB_SOURCES_HASH
#define AKB_SOURCES_HASH "unknown"
#endif
const char* akb_sources_hash(void) { return AKB_SOURCES_HASH; }
int akb_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int akb_reserved_cu_mask(int reserve, int ncu, uint32_t* mask) {
    clear_error();
    AKB_REQUIRE(mask, "null pointer");
    AKB_REQUIRE(ncu >= 256 && ncu % 32 == 0, "CU count not a multiple of 32 of at least 256");
    AKB_REQUIRE(reserve >= 0 && reserve <= 128 && reserve % 8 == 0, "reserve must be a multiple of 8 up to 128");
    for (int w = 0; w < ncu / 32; ++w) mask[w] = 0xffffffffu;
    // bits x*32 + (x + o_k) % 32 (x < 8, k < reserve/8, fixed offsets o_k = 8 (k % 4) + k / 4):
    // per XCD the same count whether the driver maps mask bits to XCDs in blocks of 32 or
    // round-robin (bit % 8): over x, (x + o_k) % 8 takes every residue once
    for (int x = 0; x < 8; ++x)
        for (int k = 0; k < reserve / 8; ++k) {
            const int b = x * 32 + (x + 8 * (k % 4) + k / 4) % 32;
            mask[b / 32] &= ~(1u << (b % 32));
        }
    return AKB_OK;
}

}  // extern "C"

namespace {
// reserved streams still alive: destroyed when the library unloads (the C runtime's exit, after
// the interpreter's own teardown has freed every tensor that recorded work on them, and before
// the HIP runtime's teardown, which this library depends on and so outlives it)
struct ReservedStreams {
    std::vector<hipStream_t> live;
    ~ReservedStreams() {
        for (hipStream_t s : live) (void)hipStreamDestroy(s);
    }
};
ReservedStreams& reserved_streams() {
    static ReservedStreams r;
    return r;
}
}  // namespace

extern "C" {

int akb_stream_create_reserved(int reserve, void** stream) {
    clear_error();
    AKB_REQUIRE(stream, "null pointer");
    int dev = 0, ncu = 0;
    AKB_HIP_CHECK(hipGetDevice(&dev));
    AKB_HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    AKB_REQUIRE(ncu >= 256 && ncu % 32 == 0, "CU count not a multiple of 32 of at least 256");
    std::vector<uint32_t> mask((size_t)ncu / 32);
    if (int st = akb_reserved_cu_mask(reserve, ncu, mask.data())) return st;
    hipStream_t st = nullptr;
    AKB_HIP_CHECK(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
    reserved_streams().live.push_back(st);
    *stream = st;
    return AKB_OK;
}

int akb_stream_destroy(void* stream) {
    clear_error();
    if (!stream) return AKB_OK;
    auto& v = reserved_streams().live;
    for (size_t i = 0; i < v.size(); ++i)
        if (v[i] == (hipStream_t)stream) {
            v.erase(v.begin() + (int64_t)i);
            break;
        }
    AKB_HIP_CHECK(hipStreamDestroy((hipStream_t)stream));
    return AKB_OK;
}

int akb_isect_f64(const double coeffs[10], const double* dir, int64_t dir_ld, int64_t dir_inc,
                  const double* org, int64_t org_ld, int64_t org_inc, int negative, int64_t n,
                  double* out, int64_t out_ld, int32_t* flags, void* stream) {
    clear_error();
    AKB_REQUIRE(coeffs && dir && org && out && flags, "null pointer");
    AKB_REQUIRE(n >= 0, "n < 0");
    if (n == 0) return AKB_OK;
    k_isect<<<grid_for(n, 1, kStreamGridCap), kBlock, 0, (hipStream_t)stream>>>(
        quadric_from(coeffs), v3in(dir, dir_ld, dir_inc), v3in(org, org_ld, org_inc), negative, n,
        V3Out{out, out_ld}, flags);
    return launch_status("k_isect");
}

int akb_normal_f64(const double coeffs[10], const double* pt, int64_t pt_ld, int64_t pt_inc, int64_t n,
                   double* out, int64_t out_ld, int normalize, int32_t* flags, void* stream) {
    clear_error();
    AKB_REQUIRE(coeffs && pt && out && flags, "null pointer");
    AKB_REQUIRE(n >= 0, "n < 0");
    if (n == 0) return AKB_OK;
    k_normal<<<grid_for(n, 1, kStreamGridCap), kBlock, 0, (hipStream_t)stream>>>(
        quadric_from(coeffs), v3in(pt, pt_ld, pt_inc), n, V3Out{out, out_ld}, normalize, flags);
    return launch_status("k_normal");
}

int akb_reflect_f64(const double* dir, int64_t dir_ld, int64_t dir_inc, const double* nrm,
                    int64_t nrm_ld, int64_t nrm_inc, int64_t n, double* out, int64_t out_ld,
                    int normalize, int32_t* flags, void* stream) {
    clear_error();
    AKB_REQUIRE(dir && nrm && out && flags, "null pointer");
    AKB_REQUIRE(n >= 0, "n < 0");
    if (n == 0) return AKB_OK;
    k_reflect<<<grid_for(n, 1, kStreamGridCap), kBlock, 0, (hipStream_t)stream>>>(
        v3in(dir, dir_ld, dir_inc), v3in(nrm, nrm_ld, nrm_inc), n, V3Out{out, out_ld}, normalize,
        flags);
    return launch_status("k_reflect");
}

int akb_normalize_f64(const double* v, int64_t v_ld, int64_t v_inc, int64_t n, double* out,
                      int64_t out_ld, int32_t* flags, void* stream) {
    clear_error();
    AKB_REQUIRE(v && out && flags, "null pointer");
    AKB_REQUIRE(n >= 0, "n < 0");
    if (n == 0) return AKB_OK;
    k_normalize<<<grid_for(n, 1, kStreamGridCap), kBlock, 0, (hipStream_t)stream>>>(v3in(v, v_ld, v_inc), n,
                                                                 V3Out{out, out_ld}, flags);
    return launch_status("k_normalize");
}

int akb_plane_isect_f64(const double ghij[4], const double* dir, int64_t dir_ld, int64_t dir_inc,
                        const double* org, int64_t org_ld, int64_t org_inc, int64_t n, double* out,
                        int64_t out_ld, void* stream) {
    clear_error();
    AKB_REQUIRE(ghij && dir && org && out, "null pointer");
    AKB_REQUIRE(n >= 0, "n < 0");
    if (n == 0) return AKB_OK;
    k_plane<<<grid_for(n, 1, kStreamGridCap), kBlock, 0, (hipStream_t)stream>>>(
        ghij[0], ghij[1], ghij[2], ghij[3], v3in(dir, dir_ld, dir_inc), v3in(org, org_ld, org_inc), n,
        V3Out{out, out_ld});
    return launch_status("k_plane");
}

int akb_seglen_f64(const double* a, int64_t a_ld, int64_t a_inc, const double* b, int64_t b_ld,
                   int64_t b_inc, int64_t n, double* out, void* stream) {
    clear_error();
    AKB_REQUIRE(a && b && out, "null pointer");
    AKB_REQUIRE(n >= 0, "n < 0");
    if (n == 0) return AKB_OK;
    k_seglen<<<grid_for(n, 1, kStreamGridCap), kBlock, 0, (hipStream_t)stream>>>(v3in(a, a_ld, a_inc),
                                                              v3in(b, b_ld, b_inc), n, out);
    return launch_status("k_seglen");
}

int akb_rotate_f64(const double ry[9], const double rz[9], const double center[3], const double* v,
                   int64_t v_ld, int64_t v_inc, int64_t n, double* out, int64_t out_ld, void* stream) {
    clear_error();
    AKB_REQUIRE(ry && rz && v && out, "null pointer");
    AKB_REQUIRE(n >= 0, "n < 0");
    if (n == 0) return AKB_OK;
    Mat3 Ry, Rz;
    for (int k = 0; k < 9; ++k) {
        Ry.m[k] = ry[k];
        Rz.m[k] = rz[k];
    }
    const int shift = center != nullptr;
    k_rotate<<<grid_for(n, 1, kStreamGridCap), kBlock, 0, (hipStream_t)stream>>>(
        Ry, Rz, shift ? center[0] : 0.0, shift ? center[1] : 0.0, shift ? center[2] : 0.0, shift,
        v3in(v, v_ld, v_inc), n, V3Out{out, out_ld});
    return launch_status("k_rotate");
}

int akb_fill_nan_f64(double* out, int64_t ld, int rows, int64_t n, void* stream) {
    clear_error();
    AKB_REQUIRE(out && rows >= 0 && n >= 0, "bad fill arguments");
    if (n == 0 || rows == 0) return AKB_OK;
    k_fill_nan<<<grid_for(n, 1, kStreamGridCap), kBlock, 0, (hipStream_t)stream>>>(out, ld, rows, n);
    return launch_status("k_fill_nan");
}

int64_t akb_chain_desc_size(void) { return (int64_t)sizeof(akb_chain_desc); }



// magic numbers for unsigned 32-bit division by d >= 2: l = ceil(log2 d),
// m' = floor(2^32 (2^l - d) / d) + 1 (Granlund & Montgomery 1994, fig. 4.1)
static void div_magic(uint32_t d, uint32_t* mul, uint32_t* shift) {
    if (d <= 1) {
        *mul = 0;
        *shift = 0;
        return;
    }
    uint32_t l = 0;
    while ((1ULL << l) < d) ++l;
    *mul = (uint32_t)((((1ULL << l) - d) << 32) / d + 1);
    *shift = l;
}

// validate a chain descriptor and form the kernel arguments (AKB_OK, or an error with n_rays == 0
// reported as AKB_OK and *empty set)
static int chain_args_from(const akb_chain_desc* d, ChainArgs& a, bool& empty) {
    empty = false;
    AKB_REQUIRE(d != nullptr, "null descriptor");
    AKB_REQUIRE(d->n_mirrors >= 0 && d->n_mirrors <= AKB_MAX_MIRRORS, "n_mirrors out of range");
    AKB_REQUIRE(d->n_rays >= 0, "n_rays < 0");
    AKB_REQUIRE(d->flags != nullptr, "flags is null");
    const bool grid = d->dir == nullptr;
    if (grid) {
        AKB_REQUIRE(d->tan_h && d->tan_v && d->n_h > 0 && d->n_v > 0, "grid tables missing");
        AKB_REQUIRE(d->ray0 >= 0 && d->ray0 + d->n_rays <= d->n_h * d->n_v,
                    "shard exceeds the ray grid");
        AKB_REQUIRE(d->n_h * d->n_v < (1LL << 32), "ray grid beyond 2^32 rays");
        AKB_REQUIRE(d->n_h < (1LL << 29) && d->n_v < (1LL << 29), "angle tables beyond 2^29 entries");
    }
    if (d->samp_v) AKB_REQUIRE(grid && d->samp_v_col >= 0 && d->samp_v_col < d->n_h, "bad samp_v_col");
    if (d->pert_h)
        AKB_REQUIRE(grid && d->pert_v && d->opl && d->pert_terms > 0 && d->pert_terms <= 8,
                    "OPL perturbation needs grid rays, opl and 1..8 terms");
    const bool sink = d->sink.nq > 0;
    if (sink) {
        AKB_REQUIRE(d->sink.nq == 5 && d->sink.n == d->n_rays && d->sink.leaf_sum && d->sink.leaf_cnt &&
                        d->sink.tail, "chain sink must be a 5-quantity sink over n_rays");
        AKB_REQUIRE(d->hits == nullptr, "per-mirror hits are written by the chain without a sink");
    }
    a = ChainArgs{};
    if (d->n_rays == 0) {
        empty = true;
        return AKB_OK;
    }
    a.K = d->n_mirrors;
    for (int k = 0; k < d->n_mirrors; ++k) {
        const double* c = d->coeffs[k];
        a.q[k] = CMirror{c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], c[8], c[9],
                         2.0 * c[0], 2.0 * c[1], 2.0 * c[2], d->negative[k] ? -1.0 : 1.0};
        // the sparse kinds need the constant term of the vanishing gradient component to be +0.0
        if (c[1] == 0.0 && c[3] == 0.0 && c[5] == 0.0 && c[7] == 0.0 && !std::signbit(c[7]))
            a.kind[k] = kKindYFree;
        else if (c[2] == 0.0 && c[4] == 0.0 && c[5] == 0.0 && c[8] == 0.0 && !std::signbit(c[8]))
            a.kind[k] = kKindZFree;
        else
            a.kind[k] = kKindGeneral;
    }
    for (int k = 0; k < 4; ++k) a.det[k] = d->det_ghij[k];
    a.dir = d->dir;
    a.dir_ld = d->dir_ld;
    a.dir_inc = d->dir_inc;
    a.tan_h = d->tan_h;
    a.tan_v = d->tan_v;
    a.n_h = grid ? (uint32_t)d->n_h : 1u;
    a.n_v = grid ? (uint32_t)d->n_v : 1u;
    div_magic(a.n_h, &a.div_mul, &a.div_shift);
    a.g0 = grid ? d->ray0 : 0;
    a.g_stride = 1;
    a.n = d->n_rays;
    a.org = d->org;
    a.org_ld = d->org_ld;
    a.org_inc = d->org_inc;
    for (int k = 0; k < 3; ++k) a.src[k] = d->src[k];
    // mirror_step's kOrigin conditions: the rays leave (+0, +0, +0), g of mirror 0 is far from
    // underflow against l (l > 0 for grid rays) and j of mirror 0 is non-zero
    a.origin0 = d->org == nullptr && d->n_mirrors > 0 && d->src[0] == 0.0 && d->src[1] == 0.0 && d->src[2] == 0.0 &&
                !std::signbit(d->src[0]) && !std::signbit(d->src[1]) && !std::signbit(d->src[2]) &&
                std::fabs(d->coeffs[0][6]) >= 0x1p-800 && std::isfinite(d->coeffs[0][6]) && d->coeffs[0][9] != 0.0;
    a.hits = d->hits;
    a.hits_ld = d->hits_ld;
    a.last_hit = d->last_hit;
    a.last_hit_ld = d->last_hit_ld;
    a.dir_out = d->dir_out;
    a.dir_out_ld = d->dir_out_ld;
    a.det_out = d->det_out;
    a.det_out_ld = d->det_out_ld;
    a.opl = d->opl;
    a.atan_h = d->atan_h;
    a.atan_v = d->atan_v;
    a.sh_begin = d->samp_h ? d->samp_h_begin : 0;
    a.sh_end = d->samp_h ? d->samp_h_end : 0;
    a.sv_col = d->samp_v_col;
    a.samp_h = d->samp_h;
    a.samp_v = d->samp_v;
    a.flags = d->flags;
    a.sink = d->sink;
    a.pert_h = d->pert_h;
    a.pert_v = d->pert_v;
    a.pert_terms = d->pert_h ? d->pert_terms : 0;
    AKB_REQUIRE(d->copy_n >= 0 && (d->copy_n == 0 || (d->copy_src && d->copy_dst)), "bad staging copy");
    a.cp_src = d->copy_src;
    a.cp_dst = d->copy_dst;
    a.cp_n = d->copy_n;
    return AKB_OK;
}

int akb_trace_chain_f64(const akb_chain_desc* d, void* stream) {
    clear_error();
    ChainArgs a;
    bool empty;
    const int st = chain_args_from(d, a, empty);
    if (st != AKB_OK || empty) return st;
    const bool grid = d->dir == nullptr;
    const bool sink = d->sink.nq > 0;
    hipStream_t s = (hipStream_t)stream;
    const int64_t gcap = kChainGridCap;
    const unsigned gsz = grid_for(d->n_rays, 1, gcap);
    const int w = kChainWaves;
    if (sink) {
        const int64_t nseg = (d->n_rays + kLeafSeg - 1) / kLeafSeg;
        const unsigned gs = (unsigned)(nseg < gcap ? nseg : gcap);
        if (grid && d->opl)
            launch_chain<true, true, true>(w, gs, s, a);
        else if (grid)
            launch_chain<true, false, true>(w, gs, s, a);
        else if (d->opl)
            launch_chain<false, true, true>(w, gs, s, a);
        else
            launch_chain<false, false, true>(w, gs, s, a);
        return launch_status("k_chain_sink");
    }
    if (grid) {
        if (d->opl)
            launch_chain<true, true, false>(w, gsz, s, a);
        else
            launch_chain<true, false, false>(w, gsz, s, a);
    } else {
        if (d->opl)
            launch_chain<false, true, false>(w, gsz, s, a);
        else
            launch_chain<false, false, false>(w, gsz, s, a);
    }
    return launch_status("k_chain");
}

// Kernel arguments of a batched launch travel through pinned host memory: a small ring of slots,
// each reused only after the event recorded behind its last copy has completed (the copy must not
// read a slot the next call is refilling). One ring per device.
namespace {
struct ArgSlot {
    void* host = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;
};
struct ArgRing {
    static constexpr int kSlots = 8;
    ArgSlot slot[kSlots];
    int next = 0;
};
std::mutex g_ring_mu;
ArgRing g_rings[64];
}  // namespace

void akb_gd_release(void);  // akb_griddata.hip: the patch-timing events and clock words

// every cache of device / pinned resources, freed while the HIP runtime is up (see the header)
void akb_release_all(void) {
    {
        std::lock_guard<std::mutex> lock(g_ring_mu);
        for (ArgRing& R : g_rings)
            for (ArgSlot& S : R.slot) {
                if (S.done) {
                    (void)hipEventSynchronize(S.done);
                    (void)hipEventDestroy(S.done);
                    S.done = nullptr;
                }
                if (S.host) (void)hipHostFree(S.host);
                S.host = nullptr;
                S.cap = 0;
            }
    }
    akb_psf_release_plans();
    akb_gd_release();
}

// copy `bytes` of host data to a fresh stream-ordered device allocation (*d_out, freed by the
// caller with hipFreeAsync on the same stream after its launch)
static int stage_args(const void* src, size_t bytes, hipStream_t s, void** d_out) {
    int dev = 0;
    AKB_HIP_CHECK(hipGetDevice(&dev));
    AKB_REQUIRE(dev >= 0 && dev < 64, "device index beyond 64");
    std::lock_guard<std::mutex> lock(g_ring_mu);
    ArgRing& R = g_rings[dev];
    ArgSlot& S = R.slot[R.next];
    R.next = (R.next + 1) % ArgRing::kSlots;
    if (S.done) AKB_HIP_CHECK(hipEventSynchronize(S.done));
    else AKB_HIP_CHECK(hipEventCreateWithFlags(&S.done, hipEventDisableTiming));
    if (S.cap < bytes) {
        if (S.host) AKB_HIP_CHECK(hipHostFree(S.host));
        S.host = nullptr;
        S.cap = 0;
        AKB_HIP_CHECK(hipHostMalloc(&S.host, bytes, hipHostMallocDefault));
        S.cap = bytes;
    }
    memcpy(S.host, src, bytes);
    AKB_HIP_CHECK(hipMallocAsync(d_out, bytes, s));
    AKB_HIP_CHECK(hipMemcpyAsync(*d_out, S.host, bytes, hipMemcpyHostToDevice, s));
    AKB_HIP_CHECK(hipEventRecord(S.done, s));
    return AKB_OK;
}

// validate a tilt's operands and fill its kernel arguments (the rotation comes from the caller)
static int tilt_args_from(TiltArgs& a, const double det1_ghij[4], const double det2_ghij[4], const double* dir,
                          const double* pt, const double* opl, int64_t ld, int64_t n, double* dir_rot, double* pt_rot,
                          double* det1, double* det2, double* total1, double* total2, const akb_leaf_sink* sink) {
    AKB_REQUIRE(det1_ghij && det2_ghij && dir && pt, "null pointer");
    AKB_REQUIRE(n >= 0 && ld >= n, "bad sizes");
    const bool use_sink = sink && sink->nq > 0;
    if (use_sink)
        AKB_REQUIRE(sink->nq == 5 && sink->n == n && sink->leaf_sum && sink->leaf_cnt && sink->tail,
                    "tilt sink must be a 5-quantity sink over n");
    for (int k = 0; k < 4; ++k) {
        a.d1[k] = det1_ghij[k];
        a.d2[k] = det2_ghij[k];
    }
    a.dir = dir;
    a.pt = pt;
    a.opl = opl;
    a.ld = ld;
    a.n = n;
    a.dir_rot = dir_rot;
    a.pt_rot = pt_rot;
    a.det1 = det1;
    a.det2 = det2;
    a.total1 = total1;
    a.total2 = total2;
    if (use_sink) a.sink = *sink;
    return AKB_OK;
}

static int launch_tilt(TiltArgs& a, const double det1_ghij[4], const double det2_ghij[4], const double* dir,
                       const double* pt, const double* opl, int64_t ld, int64_t n, double* dir_rot, double* pt_rot,
                       double* det1, double* det2, double* total1, double* total2, const akb_leaf_sink* sink,
                       void* stream) {
    const int st = tilt_args_from(a, det1_ghij, det2_ghij, dir, pt, opl, ld, n, dir_rot, pt_rot, det1, det2, total1,
                                  total2, sink);
    if (st != AKB_OK) return st;
    if (n == 0) return AKB_OK;
    if (sink && sink->nq > 0) {
        const int64_t nseg = (n + kLeafSeg - 1) / kLeafSeg;
        const unsigned gs = (unsigned)(nseg < kStreamGridCap ? nseg : kStreamGridCap);
        k_tilt_opd_sink<<<gs, kBlock, 0, (hipStream_t)stream>>>(a);
        return launch_status("k_tilt_opd_sink");
    }
    k_tilt_opd<<<grid_for(n, 1, kStreamGridCap), kBlock, 0, (hipStream_t)stream>>>(a);
    return launch_status("k_tilt_opd");
}

int akb_tilt_opd_f64(const double ry[9], const double rz[9], const double center[3],
                     const double det1_ghij[4], const double det2_ghij[4], const double* dir,
                     const double* pt, const double* opl, int64_t ld, int64_t n, double* dir_rot,
                     double* pt_rot, double* det1, double* det2, double* total1, double* total2,
                     const akb_leaf_sink* sink, void* stream) {
    clear_error();
    AKB_REQUIRE(ry && rz && center, "null pointer");
    TiltArgs a{};
    for (int k = 0; k < 9; ++k) {
        a.Ry.m[k] = ry[k];
        a.Rz.m[k] = rz[k];
    }
    for (int k = 0; k < 3; ++k) a.c[k] = center[k];
    a.params = nullptr;
    return launch_tilt(a, det1_ghij, det2_ghij, dir, pt, opl, ld, n, dir_rot, pt_rot, det1, det2, total1, total2,
                       sink, stream);
}

int akb_plane_sweep_rows_f64(const double* dir, const double* pt, int64_t ld, int64_t n, const int64_t* subset,
                             int64_t m, const double* d_plane_j, int P, const double* d_sums, double* rows,
                             void* stream) {
    clear_error();
    AKB_REQUIRE(dir && pt && d_plane_j && rows, "null pointer");
    AKB_REQUIRE(n >= 0 && ld >= n && m >= 0 && (subset || m == n), "bad sizes");
    AKB_REQUIRE(P > 0 && P <= 32767, "1..32767 planes");
    if (m == 0) return AKB_OK;
    const unsigned gx = grid_for(m, 1, kStreamGridCap / P > 0 ? kStreamGridCap / P : 1);
    k_plane_sweep<<<dim3(gx, P), kBlock, 0, (hipStream_t)stream>>>(dir, pt, ld, subset, m, d_plane_j, P, d_sums,
                                                                   (double)m, rows);
    return launch_status("k_plane_sweep");
}

int akb_plane_sweep_sink_f64(const double* dir, const double* pt, int64_t ld, int64_t n, const int64_t* subset,
                             int64_t m, const double* d_plane_j, int P, const double* d_sums,
                             const akb_leaf_sink* sink, void* stream) {
    clear_error();
    AKB_REQUIRE(dir && pt && d_plane_j && sink, "null pointer");
    AKB_REQUIRE(n >= 0 && ld >= n && m >= 0 && (subset || m == n), "bad sizes");
    AKB_REQUIRE(P > 0 && sink->nq >= 2 * P && sink->nq % (2 * kSweepGroup) == 0 && sink->n == m &&
                    sink->nan_mask == 0,
                "the sink must hold 2P quantities (padded to a multiple of 16) of m elements, no NaN skipping");
    if (m == 0) return AKB_OK;
    const int64_t nseg = (m + kLeafSeg - 1) / kLeafSeg;
    const unsigned g = (unsigned)(nseg < kStreamGridCap ? nseg : kStreamGridCap);
    AKB_REQUIRE(P <= 2048, "at most 2048 planes per sweep");
    const size_t lds = d_sums ? (size_t)(2 * P) * sizeof(double) : 0;
    k_plane_sweep_sink<<<g, kBlock, lds, (hipStream_t)stream>>>(dir, pt, ld, subset, m, d_plane_j, P, d_sums,
                                                                (double)m, *sink);
    return launch_status("k_plane_sweep_sink");
}

int akb_calc_ds_f64(const double* points, int64_t ld, int V, int H, double* d_out, void* stream) {
    clear_error();
    AKB_REQUIRE(points && d_out, "null pointer");
    AKB_REQUIRE(V >= 3 && H >= 3 && ld >= (int64_t)V * H, "calc_dS needs a grid of at least 3 x 3 points");
    const int64_t n = (int64_t)V * H;
    k_calc_ds<<<grid_for(n, 1, kStreamGridCap), kBlock, 0, (hipStream_t)stream>>>(points, ld, V, H, d_out);
    return launch_status("k_calc_ds");
}

int akb_tilt_params_f64(const double* d_sum5, const int64_t* d_cnt5, double* d_params, uint64_t* d_extent_keys,
                        int32_t* d_clear, int n_clear, void* stream) {
    clear_error();
    AKB_REQUIRE(d_sum5 && d_cnt5 && d_params, "null pointer");
    AKB_REQUIRE(n_clear >= 0 && (n_clear == 0 || d_clear), "bad clear list");
    k_tilt_params<<<1, 64, 0, (hipStream_t)stream>>>(d_sum5, d_cnt5, d_params, (unsigned long long*)d_extent_keys,
                                                      d_clear, n_clear);
    return launch_status("k_tilt_params");
}

int64_t akb_finish_params_work_bytes(const akb_leaf_sink* sink) {
    if (!sink || sink->nq <= 0 || sink->n < 0) return 0;
    const int64_t nfull = sink->n / kNpBuf;
    return (int64_t)sink->nq * (nfull + 1) * 16 + 64;
}

int akb_finish_tilt_params_f64(const akb_leaf_sink* sink, double* d_sum5, int64_t* d_cnt5, double* d_params,
                               uint64_t* d_extent_keys, int32_t* d_clear, int n_clear, void* work, void* stream) {
    clear_error();
    AKB_REQUIRE(sink && d_sum5 && d_cnt5 && d_params && work, "null pointer");
    AKB_REQUIRE(sink->nq == 5 && sink->n > 0, "the tilt's pass-2 sink: five quantities over n > 0 rays");
    AKB_REQUIRE(n_clear >= 0 && (n_clear == 0 || d_clear), "bad clear list");
    const int64_t nfull = sink->n / kNpBuf;
    AKB_REQUIRE(nfull < (1LL << 31), "too many buffers");
    double* part = (double*)work;
    long long* part_cnt = (long long*)(part + (int64_t)sink->nq * (nfull + 1));
    hipStream_t s = (hipStream_t)stream;
    const int tail = (int)(sink->n - nfull * kNpBuf);
    const int64_t nb = (nfull + kFinBPB - 1) / kFinBPB + (tail > 0 ? 1 : 0);
    if (nb > 0) {
        k_fin_buffers<<<dim3((unsigned)nb, (unsigned)sink->nq), 256, (size_t)(tail > 0 ? tail : 1) * 8, s>>>(
            *sink, nfull, part, part_cnt);
        int st = launch_status("k_fin_buffers");
        if (st) return st;
    }
    k_fin_params<<<1, 320, 0, s>>>(*sink, nfull, part, part_cnt, d_sum5, d_cnt5, d_params,
                                   (unsigned long long*)d_extent_keys, d_clear, n_clear);
    return launch_status("k_fin_params");
}

int akb_tilt_opd_dev_f64(const double* d_params, const double det1_ghij[4], const double det2_ghij[4],
                         const double* dir, const double* pt, const double* opl, int64_t ld, int64_t n,
                         double* dir_rot, double* pt_rot, double* det1, double* det2, double* total1,
                         double* total2, const akb_leaf_sink* sink, void* stream) {
    clear_error();
    AKB_REQUIRE(d_params, "null pointer");
    TiltArgs a{};
    a.params = d_params;
    return launch_tilt(a, det1_ghij, det2_ghij, dir, pt, opl, ld, n, dir_rot, pt_rot, det1, det2, total1, total2,
                       sink, stream);
}

int akb_trace_chain_batch_f64(const akb_chain_desc* descs, int n_sys, void* stream) {
    clear_error();
    AKB_REQUIRE(descs != nullptr && n_sys > 0 && n_sys <= 65535, "need 1..65535 descriptors");
    std::vector<ChainArgs> args((size_t)n_sys);
    int64_t nmax = 0;
    for (int s = 0; s < n_sys; ++s) {
        const akb_chain_desc* d = descs + s;
        bool empty = false;
        const int st = chain_args_from(d, args[s], empty);
        if (st != AKB_OK) return st;
        AKB_REQUIRE(d->dir == nullptr, "batched systems take grid rays (tan_h / tan_v)");
        AKB_REQUIRE(d->sink.nq == 0 && d->samp_h == nullptr && d->samp_v == nullptr && d->copy_n == 0,
                    "batched systems have no sink, resample picks or staging copy");
        AKB_REQUIRE((d->opl != nullptr) == (descs[0].opl != nullptr) &&
                        (d->hits != nullptr) == (descs[0].hits != nullptr),
                    "every system of a batch asks for the same opl / hits rows");
        if (empty) args[s].n = 0;
        if (args[s].n > nmax) nmax = args[s].n;
    }
    if (nmax == 0) return AKB_OK;
    hipStream_t s = (hipStream_t)stream;
    void* d_args = nullptr;
    int st = stage_args(args.data(), sizeof(ChainArgs) * args.size(), s, &d_args);
    if (st != AKB_OK) return st;
    const unsigned gx = grid_for(nmax, 1, 4096);
    const dim3 grid(gx, (unsigned)n_sys);
    const ChainArgs* A = (const ChainArgs*)d_args;
    const bool opl = descs[0].opl != nullptr, hits = descs[0].hits != nullptr;
    if (opl && hits)
        k_chain_batch<true, true><<<grid, kBlock, 0, s>>>(A);
    else if (opl)
        k_chain_batch<true, false><<<grid, kBlock, 0, s>>>(A);
    else if (hits)
        k_chain_batch<false, true><<<grid, kBlock, 0, s>>>(A);
    else
        k_chain_batch<false, false><<<grid, kBlock, 0, s>>>(A);
    st = launch_status("k_chain_batch");
    AKB_HIP_CHECK(hipFreeAsync(d_args, s));
    return st;
}

int akb_trace_chain_samples_f64(const akb_chain_desc* d, void* stream) {
    clear_error();
    AKB_REQUIRE(d != nullptr, "null descriptor");
    ChainArgs a;
    bool empty;
    const int st = chain_args_from(d, a, empty);
    if (st != AKB_OK) return st;
    AKB_REQUIRE(d->dir == nullptr && d->opl == nullptr && d->sink.nq == 0, "the picks come from grid rays of pass 1");
    AKB_REQUIRE(d->samp_h || d->samp_v, "no picks requested");
    const bool has_h = d->samp_h && d->samp_h_end > d->samp_h_begin;
    if (has_h)
        AKB_REQUIRE(d->samp_h_begin >= 0 && d->samp_h_end <= d->n_h * d->n_v, "pick range outside the grid");
    // only the picks and the flags leave these rays
    a.hits = a.last_hit = a.dir_out = a.det_out = a.opl = a.atan_h = a.atan_v = nullptr;
    a.cp_n = 0;
    a.pert_h = a.pert_v = nullptr;
    hipStream_t s = (hipStream_t)stream;
    if (has_h) {  // the middle-row range: contiguous flat indices
        ChainArgs r = a;
        r.samp_v = nullptr;
        r.g0 = d->samp_h_begin;
        r.g_stride = 1;
        r.n = d->samp_h_end - d->samp_h_begin;
        k_chain<true, false, 4><<<grid_for(r.n), kBlock, 0, s>>>(r);
        const int e = launch_status("k_chain (picks, row)");
        if (e != AKB_OK) return e;
    }
    if (d->samp_v) {  // one grid column: flat indices col, col + n_h, ...
        ChainArgs c = a;
        c.samp_h = nullptr;
        c.g0 = d->samp_v_col;
        c.g_stride = d->n_h;
        c.n = d->n_v;
        k_chain<true, false, 4><<<grid_for(c.n), kBlock, 0, s>>>(c);
        return launch_status("k_chain (picks, column)");
    }
    return AKB_OK;
}

static int chain_tilt(const akb_chain_desc* d, const double* d_params, const double det1_ghij[4],
                      const double det2_ghij[4], const double* dir, const double* pt, const double* opl, int64_t ld,
                      int64_t n, double* dir_rot, double* pt_rot, double* det1, double* det2, double* total1,
                      double* total2, const akb_leaf_sink* sink, const OpdRows* o, void* stream) {
    AKB_REQUIRE(d && d_params && sink, "null pointer");
    ChainArgs a;
    bool empty;
    int st = chain_args_from(d, a, empty);
    if (st != AKB_OK) return st;
    AKB_REQUIRE(d->dir == nullptr && d->opl == nullptr && d->sink.nq == 0,
                "the fused kernel runs pass 1: grid rays, no OPL, no sink of its own");
    AKB_REQUIRE(d->n_rays == n, "the chain and the tilt must cover the same rays");
    AKB_REQUIRE(opl != nullptr, "the fused tilt needs the pass-2 OPL row");
    AKB_REQUIRE(d->org == nullptr, "the fused pass 1 traces from a point source");
    AKB_REQUIRE(det2 && total2 && !det1 && !total1 && !dir_rot && !pt_rot,
                "the fused tilt writes the detector-2 rows only (detector 1 / rotated rays: unfused)");
    AKB_REQUIRE(!d->last_hit && !d->dir_out && !d->det_out && !d->atan_h && !d->atan_v && !d->hits && !d->samp_h &&
                    !d->samp_v,
                "the fused pass 1 writes only the flags (its picks come from akb_trace_chain_samples_f64)");
    AKB_REQUIRE(sink->nq > 0, "the tilt needs its sink");
    TiltArgs b{};
    b.params = d_params;
    st = tilt_args_from(b, det1_ghij, det2_ghij, dir, pt, opl, ld, n, dir_rot, pt_rot, det1, det2, total1, total2,
                        sink);
    if (st != AKB_OK || empty) return st;
    const int64_t nseg = (n + kLeafSeg - 1) / kLeafSeg;
    const int64_t gcap = kChainGridCap;
    const unsigned gs = (unsigned)(nseg < gcap ? nseg : gcap);
    hipStream_t s = (hipStream_t)stream;
    const OpdRows no{};
    // 22 KB of dynamic LDS beside its 18.6 KB static: three pass-1 workgroups a CU (their VGPRs
    // would allow four) leave every SIMD a wave of 128 VGPRs and 38 KB of LDS, where the faithful
    // chain's 256-thread workgroups run beside the pass instead of waiting for it to drain a CU
    constexpr size_t kPass1LdsPad = 22528;
#define AKB_CT(W)                                                  \
    if (o)                                                         \
        k_chain_tilt<W, true><<<gs, kBlock, kPass1LdsPad, s>>>(a, b, *o);     \
    else                                                           \
        k_chain_tilt<W, false><<<gs, kBlock, kPass1LdsPad, s>>>(a, b, no);
    AKB_CT(kChainWaves)
#undef AKB_CT
    return launch_status("k_chain_tilt");
}

int akb_chain_tilt_f64(const akb_chain_desc* d, const double* d_params, const double det1_ghij[4],
                       const double det2_ghij[4], const double* dir, const double* pt, const double* opl, int64_t ld,
                       int64_t n, double* dir_rot, double* pt_rot, double* det1, double* det2, double* total1,
                       double* total2, const akb_leaf_sink* sink, void* stream) {
    clear_error();
    return chain_tilt(d, d_params, det1_ghij, det2_ghij, dir, pt, opl, ld, n, dir_rot, pt_rot, det1, det2, total1,
                      total2, sink, nullptr, stream);
}

int akb_chain_tilt_opd_f64(const akb_chain_desc* d, const double* d_params, const double det1_ghij[4],
                           const double det2_ghij[4], const double* dir, const double* pt, const double* opl,
                           int64_t ld, int64_t n, double* det2, double* total2, const akb_leaf_sink* sink,
                           const double* opd_total2, const double* opd_det2, const double* d_sum5,
                           const int64_t* d_cnt5, double* dist_err2, double* wave, uint64_t* d_extent_keys,
                           void* stream) {
    clear_error();
    AKB_REQUIRE(opd_total2 && opd_det2 && d_sum5 && d_cnt5 && dist_err2 && wave && d_extent_keys,
                "the fused OPD needs the earlier run's total2, det2 and tilt sums, and writes DistError2, "
                "Wave2 and the extent keys");
    OpdRows o{};
    o.t2 = opd_total2;
    o.det2 = opd_det2;
    o.sum5 = d_sum5;
    o.cnt5 = d_cnt5;
    o.e2 = dist_err2;
    o.wave = wave;
    o.ext = (unsigned long long*)d_extent_keys;
    return chain_tilt(d, d_params, det1_ghij, det2_ghij, dir, pt, opl, ld, n, nullptr, nullptr, nullptr, det2,
                      nullptr, total2, sink, &o, stream);
}

int akb_opd_f64(const double* total1, const double* total2, const double* det2, int64_t ld, int64_t n,
                const double* d_sum5, const int64_t* d_cnt5, double* dist_err1, double* dist_err2,
                double* sph, double* wave, uint64_t* d_extent_keys, int keys_zeroed, void* stream) {
    clear_error();
    AKB_REQUIRE(n >= 0 && ld >= n, "bad sizes");
    AKB_REQUIRE(total2 && det2 && d_sum5 && d_cnt5, "total2, det2 and the tilt means are required");
    AKB_REQUIRE(!dist_err1 || total1, "dist_err1 needs total1");
    hipStream_t s = (hipStream_t)stream;
    if (d_extent_keys && !keys_zeroed) AKB_HIP_CHECK(hipMemsetAsync(d_extent_keys, 0, 4 * sizeof(uint64_t), s));
    if (n == 0) return AKB_OK;
    OpdArgs a{};
    a.t1 = total1;
    a.t2 = total2;
    a.det2 = det2;
    a.ld = ld;
    a.n = n;
    a.sum5 = d_sum5;
    a.cnt5 = d_cnt5;
    a.e1 = dist_err1;
    a.e2 = dist_err2;
    a.sph = sph;
    a.wave = wave;
    a.ext = (unsigned long long*)d_extent_keys;
    k_opd<<<grid_for(n, 1, kOpdGridCap), kBlock, 0, s>>>(a);
    return launch_status("k_opd");
}

int akb_pupil_sample_f64(const double* wave, int64_t ray0, int64_t nrays, int64_t n, int size,
                         const uint64_t* d_extent_keys, double* opd_m, double* d_pitch, void* stream) {
    clear_error();
    AKB_REQUIRE(wave && opd_m, "null pointer");
    AKB_REQUIRE(size >= 2 && n >= 2 && ray0 >= 0 && nrays >= 0 && ray0 + nrays <= n * n, "bad sizes");
    AKB_REQUIRE(!d_pitch || d_extent_keys, "pitch needs the extent keys");
    const int64_t total = (int64_t)size * size;
    k_pupil<<<grid_for(total), kBlock, 0, (hipStream_t)stream>>>(
        wave, ray0, nrays, n, size, (const unsigned long long*)d_extent_keys, opd_m, d_pitch);
    return launch_status("k_pupil");
}

}  // extern "C"

// ---- diagnostics: the trace's arithmetic shortcuts against the plain operations ----
namespace akb {
constexpr int kSelftestCols = AKB_SELFTEST_COLS;

// out row i: sqrt_cr(a), sqrt(a), div_shared(a, b), a / b, div_pos(a, b), norm3_inv's s and inv of
// (a, b, b), norm3 with 1.0 / norm3 of the same vector, atan_slope(a), OCML's atan(a), div_w(a, b)
// and div_w(1, b)
__global__ void k_selftest(const double* a, const double* b, int64_t n, double* out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double x = a[i], s = b[i];
        double* o = out + (int64_t)kSelftestCols * i;
        o[0] = sqrt_cr(x);
        o[1] = sqrt(x);
        o[2] = div_shared(x, s, 1.0 / s);
        o[3] = x / s;
        o[4] = div_pos(x, s, 1.0 / s);
        double nv, ninv;
        norm3_inv(x, s, s, nv, ninv);
        o[5] = nv;
        o[6] = ninv;
        const double v = x * x + s * s + s * s;
        o[7] = sqrt(v);
        o[8] = 1.0 / sqrt(v);
        o[9] = atan_slope(x);
        o[10] = atan(x);
        o[11] = div_w(x, s);
        o[12] = div_w(1.0, s);
    }
}
}  // namespace akb

extern "C" int akb_selftest_arith_f64(const double* a, const double* b, int64_t n, double* out, void* stream) {
    akb::clear_error();
    AKB_REQUIRE(a && b && out && n >= 0, "bad selftest arguments");
    if (n == 0) return AKB_OK;
    akb::k_selftest<<<akb::grid_for(n), akb::kBlock, 0, (hipStream_t)stream>>>(a, b, n, out);
    return akb::launch_status("k_selftest");
}

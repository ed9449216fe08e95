/*
 * akb_oracle.c — CPU restatement of the reference's ray-trace arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity checker for the HIP kernels and the timed
 * CPU baseline of bench.py ("kind": "port"). Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product path never does.
 *
 * Compiled with gcc -O2 -ffp-contract=off (see oracle/Makefile): SSE2 doubles, every product and
 * sum rounded separately, in the association order numpy evaluates the reference's expressions.
 * Pinned bit-for-bit against vectors captured from the reference itself
 * (tests/golden/make_golden.py writes the .npz fixtures, checked by tests/test_oracle_golden.py).
 *
 * Reference functions restated (Kakekakechan/AKBRaytracing):
 *   oracle_isect      mirr_ray_intersection   EllipseRaytrace3D.py:18-45; AKB_raytrace_20250312.py:444-471
 *   oracle_normal     norm_vector             EllipseRaytrace3D.py:61-71; AKB_raytrace_20250312.py:626-636
 *   oracle_reflect    reflect_ray             EllipseRaytrace3D.py:47-55; AKB_raytrace_20250312.py:501-509
 *   oracle_normalize  normalize_vector        EllipseRaytrace3D.py:57-59; AKB_raytrace_20250312.py:530-532
 *   oracle_plane      plane_ray_intersection  EllipseRaytrace3D.py:145-157; AKB_raytrace_20250312.py:873-885
 *   oracle_seglen     np.linalg.norm(b - a, axis=0)  AKB_raytrace_20250312.py:2884-2897
 *   oracle_rotate     rotate_vectors / rotate_points (dgemm FMA order)  AKB_raytrace_20250312.py:917-943
 *   oracle_np_sum     numpy add.reduce on a contiguous float64 row (8192-blocks, pairwise)
 *   oracle_huygens    compute_u_parallel      Wavecalc_raytrace_fromData_CPU0402.py:71-85
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define X(p, ld, inc, i) ((p)[(i) * (inc)])
#define Y(p, ld, inc, i) ((p)[(ld) + (i) * (inc)])
#define Z(p, ld, inc, i) ((p)[2 * (ld) + (i) * (inc)])

static void fill_nan(double* out, int64_t ld, int64_t n) {
    const double q = NAN;
    for (int64_t i = 0; i < n; ++i) out[i] = out[ld + i] = out[2 * ld + i] = q;
}

/* returns 1 when any discriminant was not > 0 and the whole output became NaN (ref :457-459) */
int oracle_isect(const double* c, const double* d, int64_t d_ld, int64_t d_inc, const double* s,
                 int64_t s_ld, int64_t s_inc, int negative, int64_t n, double* out, int64_t o_ld) {
    const double a = c[0], b = c[1], cc = c[2], dd = c[3], e = c[4], f = c[5], g = c[6], h = c[7],
                 ii = c[8], j = c[9];
    int miss = 0;
#pragma omp parallel for reduction(| : miss) schedule(static)
    for (int64_t k = 0; k < n; ++k) {
        const double l = X(d, d_ld, d_inc, k), m = Y(d, d_ld, d_inc, k), nn = Z(d, d_ld, d_inc, k);
        const double p = X(s, s_ld, s_inc, k), q = Y(s, s_ld, s_inc, k), r = Z(s, s_ld, s_inc, k);
        const double A = a * (l * l) + b * (m * m) + cc * (nn * nn) + dd * m * l + e * nn * l + f * m * nn;
        const double B = 2.0 * a * p * l + 2.0 * b * q * m + 2.0 * cc * r * nn + dd * (p * m + q * l) +
                         e * (p * nn + r * l) + f * (r * m + q * nn) + g * l + h * m + ii * nn;
        const double C = a * (p * p) + b * (q * q) + cc * (r * r) + dd * p * q + e * p * r + f * q * r +
                         g * p + h * q + ii * r + j;
        const double D = B * B - 4.0 * A * C;
        if (!(D > 0.0)) miss = 1;
        const double sq = sqrt(B * B - 4.0 * A * C);
        const double t = (negative ? (-B - sq) : (-B + sq)) / (2.0 * A);
        out[k] = t * l + p;
        out[o_ld + k] = t * m + q;
        out[2 * o_ld + k] = t * nn + r;
    }
    if (miss) fill_nan(out, o_ld, n);
    return miss;
}

/* np.linalg.norm(v, axis=0) then v / norm unless any norm == 0 (returns 1: v passed through) */
static int normalize_inplace(double* v, int64_t ld, int64_t n) {
    int zero = 0;
    double* nrm = (double*)malloc(sizeof(double) * (n > 0 ? n : 1));
#pragma omp parallel for reduction(| : zero) schedule(static)
    for (int64_t k = 0; k < n; ++k) {
        const double x = v[k], y = v[ld + k], z = v[2 * ld + k];
        nrm[k] = sqrt(x * x + y * y + z * z);
        if (nrm[k] == 0.0) zero = 1;
    }
    if (!zero) {
#pragma omp parallel for schedule(static)
        for (int64_t k = 0; k < n; ++k) {
            v[k] = v[k] / nrm[k];
            v[ld + k] = v[ld + k] / nrm[k];
            v[2 * ld + k] = v[2 * ld + k] / nrm[k];
        }
    }
    free(nrm);
    return zero;
}

int oracle_normalize(const double* v, int64_t v_ld, int64_t v_inc, int64_t n, double* out, int64_t o_ld) {
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < n; ++k) {
        out[k] = X(v, v_ld, v_inc, k);
        out[o_ld + k] = Y(v, v_ld, v_inc, k);
        out[2 * o_ld + k] = Z(v, v_ld, v_inc, k);
    }
    return normalize_inplace(out, o_ld, n);
}

int oracle_normal(const double* c, const double* pt, int64_t p_ld, int64_t p_inc, int64_t n, double* out,
                  int64_t o_ld) {
    const double a = c[0], b = c[1], cc = c[2], dd = c[3], e = c[4], f = c[5], g = c[6], h = c[7],
                 ii = c[8];
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < n; ++k) {
        const double x = X(pt, p_ld, p_inc, k), y = Y(pt, p_ld, p_inc, k), z = Z(pt, p_ld, p_inc, k);
        out[k] = 2.0 * a * x + dd * y + e * z + g;
        out[o_ld + k] = 2.0 * b * y + dd * x + f * z + h;
        out[2 * o_ld + k] = 2.0 * cc * z + e * x + f * y + ii;
    }
    return normalize_inplace(out, o_ld, n);
}

int oracle_reflect(const double* d, int64_t d_ld, int64_t d_inc, const double* nv, int64_t n_ld,
                   int64_t n_inc, int64_t n, double* out, int64_t o_ld) {
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < n; ++k) {
        const double l = X(d, d_ld, d_inc, k), m = Y(d, d_ld, d_inc, k), nn = Z(d, d_ld, d_inc, k);
        const double nx = X(nv, n_ld, n_inc, k), ny = Y(nv, n_ld, n_inc, k), nz = Z(nv, n_ld, n_inc, k);
        const double A2 = 2.0 * (l * nx + m * ny + nn * nz);
        out[k] = l - A2 * nx;
        out[o_ld + k] = m - A2 * ny;
        out[2 * o_ld + k] = nn - A2 * nz;
    }
    return normalize_inplace(out, o_ld, n);
}

void oracle_plane(const double* ghij, const double* d, int64_t d_ld, int64_t d_inc, const double* s,
                  int64_t s_ld, int64_t s_inc, int64_t n, double* out, int64_t o_ld) {
    const double g = ghij[0], h = ghij[1], ii = ghij[2], j = ghij[3];
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < n; ++k) {
        const double l = X(d, d_ld, d_inc, k), m = Y(d, d_ld, d_inc, k), nn = Z(d, d_ld, d_inc, k);
        const double p = X(s, s_ld, s_inc, k), q = Y(s, s_ld, s_inc, k), r = Z(s, s_ld, s_inc, k);
        const double t = -(g * p + h * q + ii * r + j) / (g * l + h * m + ii * nn);
        out[k] = t * l + p;
        out[o_ld + k] = t * m + q;
        out[2 * o_ld + k] = t * nn + r;
    }
}

void oracle_seglen(const double* a, int64_t a_ld, int64_t a_inc, const double* b, int64_t b_ld,
                   int64_t b_inc, int64_t n, double* out) {
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < n; ++k) {
        const double dx = X(b, b_ld, b_inc, k) - X(a, a_ld, a_inc, k);
        const double dy = Y(b, b_ld, b_inc, k) - Y(a, a_ld, a_inc, k);
        const double dz = Z(b, b_ld, b_inc, k) - Z(a, a_ld, a_inc, k);
        out[k] = sqrt(dx * dx + dy * dy + dz * dz);
    }
}

/* out = Ry @ (Rz @ (v - c)) + c (center may be NULL). numpy hands (3,3) @ (3,N) to OpenBLAS
 * dgemm, whose kernel forms each output as r0*x, then fma(r1, y, .), then fma(r2, z, .);
 * restated here with fma() so the rotation matches the reference bit for bit. */
static inline void mat3_row(const double* R, double x, double y, double z, double* o) {
    for (int i = 0; i < 3; ++i) {
        double c = R[3 * i] * x;
        c = fma(R[3 * i + 1], y, c);
        o[i] = fma(R[3 * i + 2], z, c);
    }
}

void oracle_rotate(const double* ry, const double* rz, const double* c, const double* v, int64_t v_ld,
                   int64_t v_inc, int64_t n, double* out, int64_t o_ld) {
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < n; ++k) {
        double x = X(v, v_ld, v_inc, k), y = Y(v, v_ld, v_inc, k), z = Z(v, v_ld, v_inc, k);
        if (c) {
            x = x - c[0];
            y = y - c[1];
            z = z - c[2];
        }
        double a[3], b[3];
        mat3_row(rz, x, y, z, a);
        mat3_row(ry, a[0], a[1], a[2], b);
        if (c) {
            b[0] = b[0] + c[0];
            b[1] = b[1] + c[1];
            b[2] = b[2] + c[2];
        }
        out[k] = b[0];
        out[o_ld + k] = b[1];
        out[2 * o_ld + k] = b[2];
    }
}

/* ---- numpy's float64 add.reduce over one contiguous row ---- */

static double pw_val(const double* a, int64_t i, int nan0, int64_t* cnt) {
    double v = a[i];
    if (nan0 && v != v) return 0.0;
    ++*cnt;
    return v;
}

static double pairwise(const double* a, int64_t n, int nan0, int64_t* cnt) {
    if (n < 8) {
        double res = 0.0;
        for (int64_t i = 0; i < n; ++i) res = res + pw_val(a, i, nan0, cnt);
        return res;
    }
    if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = pw_val(a, j, nan0, cnt);
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] = r[j] + pw_val(a, i + j, nan0, cnt);
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res = res + pw_val(a, i, nan0, cnt);
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    const double left = pairwise(a, n2, nan0, cnt);
    return left + pairwise(a + n2, n - n2, nan0, cnt);
}

/* np.sum(x) (nan0=0) or np.nansum-style (nan0=1); *count = summed elements */
double oracle_np_sum(const double* x, int64_t n, int nan0, int64_t* count) {
    int64_t cnt = 0;
    double acc = 0.0;
    for (int64_t b = 0; b < n; b += 8192) {
        const int64_t len = (n - b) < 8192 ? (n - b) : 8192;
        const double part = pairwise(x + b, len, nan0, &cnt);
        acc = (b == 0) ? part : acc + part;
    }
    if (count) *count = cnt;
    return acc;
}

/* compute_u_parallel: one target per iteration, numpy-sequential order over sources is not
 * reproduced (numpy sums pairwise); this is the speed baseline, checked by tolerance. */
void oracle_huygens(const double* tx, const double* ty, const double* tz, int64_t n, const double* sx,
                    const double* sy, const double* sz, const double* u, int64_t m, double k,
                    double* out) {
    const double negk = -k;
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t i = 0; i < n; ++i) {
        double ar = 0.0, ai = 0.0;
        for (int64_t j = 0; j < m; ++j) {
            const double dx = tx[i] - sx[j], dy = ty[i] - sy[j], dz = tz[i] - sz[j];
            const double r = sqrt(dx * dx + dy * dy + dz * dz);
            const double amp = 1.0 / r;
            const double ph = negk * r;
            const double fr = amp * cos(ph), fi = amp * sin(ph);
            ar += fr * u[2 * j] - fi * u[2 * j + 1];
            ai += fr * u[2 * j + 1] + fi * u[2 * j];
        }
        out[2 * i] = ar;
        out[2 * i + 1] = ai;
    }
}

/* calc_dS (AKB_raytrace_20250312.py:13418-13473): the triangle norms are np.linalg.norm of a
 * 3-vector, which numpy hands to BLAS ddot; OpenBLAS accumulates x0*x0, then fma(x1, x1, .),
 * then fma(x2, x2, .) — restated with explicit fma() (measured: bit-identical on the fixture). */
static double tri_area(const double* p, const double* a, const double* b) {
    double e1[3], e2[3];
    for (int k = 0; k < 3; ++k) {
        e1[k] = a[k] - p[k];
        e2[k] = b[k] - p[k];
    }
    const double c0 = e1[1] * e2[2] - e1[2] * e2[1];
    const double c1 = e1[2] * e2[0] - e1[0] * e2[2];
    const double c2 = e1[0] * e2[1] - e1[1] * e2[0];
    return sqrt(fma(c2, c2, fma(c1, c1, c0 * c0))) / 2;
}

void oracle_calc_ds(const double* pts, int64_t ld, int V, int H, double* out) {
    for (int i0 = 0; i0 < V; ++i0)
        for (int j0 = 0; j0 < H; ++j0) {
            const int i = i0 < 1 ? 1 : (i0 > V - 2 ? V - 2 : i0);
            const int j = j0 < 1 ? 1 : (j0 > H - 2 ? H - 2 : j0);
            double q[5][3];
            const int ii[5] = {i, i, i - 1, i, i + 1}, jj[5] = {j, j + 1, j, j - 1, j};  /* p, right, up, left, down */
            for (int t = 0; t < 5; ++t)
                for (int k = 0; k < 3; ++k) q[t][k] = pts[k * ld + (int64_t)ii[t] * H + jj[t]];
            double s = 0.0;
            s += tri_area(q[0], q[1], q[2]);
            s += tri_area(q[0], q[2], q[3]);
            s += tri_area(q[0], q[3], q[4]);
            s += tri_area(q[0], q[4], q[1]);
            out[(int64_t)i0 * H + j0] = s;
        }
}

int oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void oracle_set_threads(int t) {
#ifdef _OPENMP
    if (t > 0) omp_set_num_threads(t);
#else
    (void)t;
#endif
}

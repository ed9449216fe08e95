// AddressSanitizer + UndefinedBehaviorSanitizer run of the library's host code and the oracle's C
// restatement (SURVEY.md §5 "sanitizers"). Built and run by tests/test_sanitize.py:
//
//   hipcc -O1 -g -fsanitize=address,undefined -fno-gpu-sanitize  host_asan_driver.cpp
//         akbraytracing_amd/csrc/akb_host.cpp akbraytracing_amd/csrc/akb_gd_host.cpp
//         akbraytracing_amd/csrc/akb_affine_host.cpp  (+ oracle C)
//
// Host-only code (no kernel launches): the equal-angle resample (akb_resample_f64: numpy linspace
// and interp restated, scipy's stable sort), the griddata pocket triangulation (akb_gd_pockets:
// hull, fixed-capacity triangle and chord arrays) and the oracle's primitives, sums and calc_dS,
// over random, ragged, NaN and degenerate inputs. Any memory error or UB aborts the process.
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <string>
#include <vector>

#include "../../include/akb_raytrace.h"

namespace akb {
static std::string g_err;
void set_error(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}
void clear_error() { g_err.clear(); }
}  // namespace akb

extern "C" {
int oracle_isect(const double* c, const double* d, int64_t d_ld, int64_t d_inc, const double* s, int64_t s_ld,
                 int64_t s_inc, int negative, int64_t n, double* out, int64_t o_ld);
int oracle_normal(const double* c, const double* pt, int64_t p_ld, int64_t p_inc, int64_t n, double* out,
                  int64_t o_ld);
int oracle_reflect(const double* d, int64_t d_ld, int64_t d_inc, const double* nv, int64_t n_ld, int64_t n_inc,
                   int64_t n, double* out, int64_t o_ld);
double oracle_np_sum(const double* x, int64_t n, int nan0, int64_t* count);
void oracle_calc_ds(const double* pts, int64_t ld, int V, int H, double* out);
}

static std::mt19937_64 rng(20261016);
static double unif(double a, double b) { return std::uniform_real_distribution<double>(a, b)(rng); }

static int resample_cases() {
    int ok = 0, refused = 0;
    for (int t = 0; t < 3000; ++t) {
        const int64_t n = 1 + (int64_t)(rng() % 700);
        std::vector<double> x(n), y(n), out(n);
        const int kind = t % 5;
        for (int64_t i = 0; i < n; ++i) {
            x[i] = kind == 1 ? unif(-1, 1) : (double)i * 1e-6 + unif(0, 1e-9);
            y[i] = unif(-1e-3, 1e-3);
        }
        if (kind == 2 && n > 2) x[rng() % n] = NAN;
        if (kind == 3) for (auto& v : x) v = 0.5;          // all equal: degenerate linspace
        if (kind == 4 && n > 1) std::swap(x[0], x[n - 1]);  // ends swapped: out-of-range picks
        const int st = akb_resample_f64(x.data(), y.data(), n, out.data());
        (st == 0 ? ok : refused)++;
    }
    printf("resample: %d ok, %d refused\n", ok, refused);
    return ok > 0;
}

static int pocket_case(int nv, int nh, int warp, bool cut_corner) {
    std::vector<double> X((size_t)nv * nh), Y((size_t)nv * nh);
    for (int i = 0; i < nv; ++i)
        for (int j = 0; j < nh; ++j) {
            const double u = -1 + 2.0 * j / (nh - 1), v = -1 + 2.0 * i / (nv - 1);
            double x = u, y = v;
            if (warp == 1) {
                x = u * 1e-4 + 3e-6 * v * v - 2e-6 * u * v + 1e-6 * v * v * v;
                y = v * 1.3e-4 + 4e-6 * u * u + 1e-6 * u * u * u;
            } else if (warp == 2) {
                x = u + 0.05 * v + 0.03 * (u + 0.3) * (u + 0.3);
                y = 0.8 * v - 0.04 * (v - 0.2) * u + 0.02 * u * u * u;
            }
            X[(size_t)i * nh + j] = x;
            Y[(size_t)i * nh + j] = y;
        }
    if (cut_corner) X[0] = Y[0] = -0.5;
    // the boundary ring: top row, right column, bottom row reversed, left column reversed
    std::vector<int64_t> r;
    for (int j = 0; j < nh - 1; ++j) r.push_back(j);
    for (int i = 0; i < nv - 1; ++i) r.push_back((int64_t)i * nh + nh - 1);
    for (int j = nh - 1; j > 0; --j) r.push_back((int64_t)(nv - 1) * nh + j);
    for (int i = nv - 1; i > 0; --i) r.push_back((int64_t)i * nh);
    const int cap = (int)r.size();
    std::vector<double> rx(cap), ry(cap);
    for (int k = 0; k < cap; ++k) {
        rx[k] = X[r[k]];
        ry[k] = Y[r[k]];
    }
    // exactly-sized outputs: any overrun is a heap error under ASan
    std::vector<int32_t> tri(3 * (size_t)cap), nbr(3 * (size_t)cap), edge(cap), xptr(cap + 1), xidx(6 * (size_t)cap);
    int32_t n = 0;
    return akb_gd_pockets(rx.data(), ry.data(), nv, nh, cap, &n, tri.data(), nbr.data(), edge.data(), xptr.data(),
                          xidx.data());
}

// extract_affine_square_region's host steps (akb_affine_host.cpp) on random masks: contours into
// exactly-sized buffers (a too-small capacity must be refused, not overrun), polygons of every
// contour at several tolerances, the affine solve and inverse
static int affine_cases() {
    int contours = 0, refused = 0;
    for (int t = 0; t < 300; ++t) {
        const int rows = 1 + (int)(rng() % 40), cols = 1 + (int)(rng() % 40);
        std::vector<uint8_t> m((size_t)rows * cols);
        const int dens = (int)(rng() % 100);
        for (auto& v : m) v = (int)(rng() % 100) < dens ? 255 : 0;
        int64_t nxy = 0;
        int32_t nc = 0;
        int32_t probe_xy[2], probe_off[1];
        if (akb_external_contours(m.data(), rows, cols, 0, probe_xy, &nxy, 0, probe_off, &nc) != 0) ++refused;
        std::vector<int32_t> xy(2 * (size_t)(nxy > 0 ? nxy : 1)), offs((size_t)nc + 1);
        if (akb_external_contours(m.data(), rows, cols, nxy, xy.data(), &nxy, nc + 1, offs.data(), &nc) != 0) return 0;
        contours += nc;
        for (int c = 0; c < nc; ++c) {
            const int32_t k = offs[c + 1] - offs[c];
            std::vector<int32_t> out(2 * (size_t)k);
            int32_t nout = 0;
            for (double eps : {0.0, 0.5, 2.0, 50.0})
                if (akb_approx_poly_dp(xy.data() + 2 * (size_t)offs[c], k, eps, 1, out.data(), &nout) != 0 && k > 1)
                    ++refused;  // coincident slice ends (a one-pixel-wide spur) are refused, as cv2 asserts
        }
    }
    for (int t = 0; t < 200; ++t) {
        float src[6], dst[6];
        for (int i = 0; i < 6; ++i) {
            src[i] = (float)unif(-50, 300);
            dst[i] = (float)unif(-10, 260);
        }
        if (t % 50 == 0) src[4] = src[0], src[5] = src[1];  // repeated point: refused
        double M[6], iM[6];
        if (akb_affine_from_points(src, dst, M) == 0) akb_affine_invert(M, iM);
    }
    printf("affine: %d contours, %d refused\n", contours, refused);
    return contours > 0;
}

static int oracle_cases() {
    const int64_t n = 1021;
    std::vector<double> d(3 * n), s(3 * n), out(3 * n), nrm(3 * n), ref(3 * n);
    for (int64_t i = 0; i < n; ++i) {
        d[i] = 1.0;
        d[n + i] = unif(-1e-3, 1e-3);
        d[2 * n + i] = unif(-1e-3, 1e-3);
    }
    const double c[10] = {1.0 / (72.98 * 72.98), 0, -1.0 / (0.26 * 0.26), 0, 0, 0, -0.02, 0, 0, -0.5};
    oracle_isect(c, d.data(), n, 1, s.data(), n, 1, 0, n, out.data(), n);
    oracle_normal(c, out.data(), n, 1, n, nrm.data(), n);
    oracle_reflect(d.data(), n, 1, nrm.data(), n, 1, n, ref.data(), n);
    int64_t cnt = 0;
    double acc = 0;
    for (int64_t m : {0L, 1L, 7L, 8L, 129L, 8191L, 8192L, 20000L}) {
        std::vector<double> x((size_t)m);
        for (auto& v : x) v = unif(-1, 1);
        if (m > 3) x[1] = NAN;
        acc += oracle_np_sum(x.data(), m, 1, &cnt);
    }
    std::vector<double> pts(3 * 17 * 13), ds(17 * 13);
    for (auto& v : pts) v = unif(0, 1);
    oracle_calc_ds(pts.data(), 17 * 13, 17, 13, ds.data());
    printf("oracle: ok (%g)\n", acc + ds[5] + ref[7]);
    return 1;
}

int main() {
    int good = resample_cases();
    int st = 0;
    for (int warp = 0; warp < 3; ++warp)
        for (int sz : {2, 3, 5, 17, 65, 129}) {
            st = pocket_case(sz, sz + (warp == 2 ? 7 : 0), warp, false);
            if (st != 0 && warp != 0) {
                printf("pockets refused a valid lattice (%d, %d): %d\n", sz, warp, st);
                return 2;
            }
        }
    st = pocket_case(20, 20, 0, true);
    printf("pockets: cut corner -> %d (refused as expected: %s)\n", st, st != 0 ? "yes" : "no");
    if (st == 0) return 3;
    good &= oracle_cases();
    good &= affine_cases();
    fflush(stdout);
    return good ? 0 : 1;
}

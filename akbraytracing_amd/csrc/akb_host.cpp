// Host-side pieces of the hot path that stay on the CPU by design (no device work).
//
// akb_resample_f64: the equal-angle resample between the two passes of the drivers
// (AKB_raytrace_20250312.py:2861-2870, KB_debug :11020-11030):
//
//     out = np.linspace(sep[0], sep[-1], n)
//     new = interp1d(sep, rand, kind='linear')(out)
//
// scipy 1.15's interp1d(kind='linear') on 1-D float64 data sorts x with a stable mergesort,
// checks bounds (ValueError) and hands over to np.interp, so this restates numpy 2.2's linspace
// and interp (compiled C) operation by operation. The arctan that turns the exit slopes into
// `sep` and the tan of the result stay numpy calls in the caller: numpy dispatches them to its
// own SIMD kernels on AVX-512 hosts, which are not libm's, and the tables must be numpy's bits.
#include <math.h>

#include <algorithm>
#include <numeric>
#include <vector>

#include "akb_common.h"

namespace {

// numpy.linspace(start, stop, n), endpoint=True, float64
void np_linspace(double start, double stop, int64_t n, double* y) {
    if (n <= 0) return;
    const double delta = stop - start;
    if (n == 1) {
        y[0] = 0.0 * delta + start;
        return;
    }
    const double div = (double)(n - 1);
    const double step = delta / div;
    if (step == 0.0) {
        for (int64_t i = 0; i < n; ++i) y[i] = ((double)i / div) * delta + start;
    } else {
        for (int64_t i = 0; i < n; ++i) y[i] = (double)i * step + start;
    }
    y[n - 1] = stop;
}

// numpy's binary_search_with_guess (numpy/_core/src/multiarray/compiled_base.c): for sorted xp the
// last j with xp[j] <= key, -1 below the range, len above it; O(1) when consecutive keys are close
int64_t np_search_with_guess(double key, const double* arr, int64_t len, int64_t guess) {
    constexpr int64_t kCache = 8;  // LIKELY_IN_CACHE_SIZE
    int64_t imin = 0, imax = len;
    if (key > arr[len - 1]) return len;
    if (key < arr[0]) return -1;
    if (len <= 4) {
        int64_t i = 1;
        while (i < len && key >= arr[i]) ++i;
        return i - 1;
    }
    if (guess > len - 3) guess = len - 3;
    if (guess < 1) guess = 1;
    if (key < arr[guess]) {
        if (key < arr[guess - 1]) {
            imax = guess - 1;
            if (guess > kCache && key >= arr[guess - kCache]) imin = guess - kCache;
        } else {
            return guess - 1;
        }
    } else {
        if (key < arr[guess + 1]) return guess;
        if (key < arr[guess + 2]) return guess + 1;
        imin = guess + 2;
        if (guess < len - kCache - 1 && key < arr[guess + kCache]) imax = guess + kCache;
    }
    while (imin < imax) {
        const int64_t imid = imin + ((imax - imin) >> 1);
        if (key >= arr[imid])
            imin = imid + 1;
        else
            imax = imid;
    }
    return imin - 1;
}

// numpy.interp(x, xp, fp) with the default left/right (fp[0], fp[-1]), float64
void np_interp(const double* x, int64_t nx, const double* xp, const double* fp, int64_t len, double* out) {
    const double lval = fp[0], rval = fp[len - 1];
    if (len == 1) {
        for (int64_t i = 0; i < nx; ++i) {
            const double v = x[i];
            out[i] = v < xp[0] ? lval : (v > xp[0] ? rval : fp[0]);
        }
        return;
    }
    std::vector<double> slopes;
    const bool pre = len <= nx;  // numpy pre-computes the slopes when there are few of them
    if (pre) {
        slopes.resize(len - 1);
        for (int64_t i = 0; i < len - 1; ++i) slopes[i] = (fp[i + 1] - fp[i]) / (xp[i + 1] - xp[i]);
    }
    int64_t j = 0;
    for (int64_t i = 0; i < nx; ++i) {
        const double v = x[i];
        if (v != v) {
            out[i] = v;
            continue;
        }
        j = np_search_with_guess(v, xp, len, j);
        if (j == -1) {
            out[i] = lval;
        } else if (j == len) {
            out[i] = rval;
        } else if (j == len - 1) {
            out[i] = fp[j];
        } else if (xp[j] == v) {
            out[i] = fp[j];
        } else {
            const double slope = pre ? slopes[j] : (fp[j + 1] - fp[j]) / (xp[j + 1] - xp[j]);
            double r = slope * (v - xp[j]) + fp[j];
            if (r != r) {
                r = slope * (v - xp[j + 1]) + fp[j + 1];
                if (r != r && fp[j] == fp[j + 1]) r = fp[j];
            }
            out[i] = r;
        }
    }
}

}  // namespace

using namespace akb;

extern "C" {

int akb_resample_f64(const double* angle_sep, const double* rand, int64_t n, double* out) {
    clear_error();
    AKB_REQUIRE(angle_sep && rand && out, "null pointer");
    AKB_REQUIRE(n > 0, "empty resample");
    std::vector<double> xnew(n), xs(n), ys(n);
    np_linspace(angle_sep[0], angle_sep[n - 1], n, xnew.data());
    // stable sort with NaN last (numpy's mergesort order); the usual monotone samples are the
    // identity (non-decreasing) or a reversal (strictly decreasing) without sorting
    std::vector<int64_t> ind(n);
    bool asc = angle_sep[0] == angle_sep[0], desc = asc;
    for (int64_t i = 1; i < n && (asc || desc); ++i) {
        const double a = angle_sep[i - 1], b = angle_sep[i];
        asc = asc && a <= b;
        desc = desc && a > b;
    }
    if (asc) {
        std::iota(ind.begin(), ind.end(), (int64_t)0);
    } else if (desc) {
        for (int64_t i = 0; i < n; ++i) ind[i] = n - 1 - i;
    } else {
        std::iota(ind.begin(), ind.end(), (int64_t)0);
        std::stable_sort(ind.begin(), ind.end(), [&](int64_t a, int64_t b) {
            const double u = angle_sep[a], v = angle_sep[b];
            return u < v || (v != v && u == u);
        });
    }
    for (int64_t i = 0; i < n; ++i) {
        xs[i] = angle_sep[ind[i]];
        ys[i] = rand[ind[i]];
    }
    for (int64_t i = 0; i < n; ++i) {
        if (xnew[i] < xs[0] || xnew[i] > xs[n - 1]) {
            set_error("A value in x_new is outside the interpolation range.");
            return AKB_E_INVALID;
        }
    }
    np_interp(xnew.data(), n, xs.data(), ys.data(), n, out);
    return AKB_OK;
}

}  // extern "C"

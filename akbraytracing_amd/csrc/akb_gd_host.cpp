// Host half of the structured Delaunay triangulation used by the device griddata (akb_griddata.hip).
//
// griddata(points, values, xi, method='cubic') (scipy 1.15, called at AKB_raytrace_20250312.py:3673
// and :3689) triangulates the scattered points with qhull's Delaunay. The points here are the
// detector hits of an n_v x n_h ray grid, a smoothly deformed lattice: its Delaunay triangulation
// is every grid cell split by the diagonal that passes the in-circle test (the device does that)
// plus the "pockets" between the grid's boundary ring and its convex hull. This file triangulates
// the pockets: hull of the ring (Andrew's monotone chain, collinear and rounding-level collinear
// points kept), then, for every
// hull edge (p, q) that skips ring points, the Delaunay triangle on its inner side - the chain
// point seeing (p, q) under the largest angle (its circumcircle holds no other chain point) - and
// the same for the two sub-chains it leaves. The device checks the result is locally Delaunay
// against the cell triangles it borders.
#include <math.h>
#include <stdlib.h>
#include <stdint.h>

#include <immintrin.h>

#include <algorithm>
#include <functional>
#include <utility>
#include <vector>

#include "akb_common.h"

namespace {

struct Ring {
    int nv, nh;
    int64_t L;
    int64_t vertex(int64_t r) const {  // ring position -> global vertex id (row-major iv * nh + ih)
        r %= L;
        const int64_t a = nh - 1, b = nv - 1;
        if (r < a) return r;                                        // bottom row, ih = r
        if (r < a + b) return (r - a) * nh + (nh - 1);              // right column, iv = r - a
        if (r < 2 * a + b) return (int64_t)(nv - 1) * nh + (nh - 1 - (r - a - b));  // top row
        return (int64_t)(nv - 1 - (r - 2 * a - b)) * nh;           // left column
    }
    bool corner(int64_t r) const {
        r %= L;
        const int64_t a = nh - 1, b = nv - 1;
        return r == 0 || r == a || r == a + b || r == 2 * a + b;
    }
};

double cross3(const double* x, const double* y, int64_t o, int64_t a, int64_t b) {
    return (x[a] - x[o]) * (y[b] - y[o]) - (y[a] - y[o]) * (x[b] - x[o]);
}

// a strict right turn o -> a -> b, beyond rounding: qhull merges the slivers that rounding-level
// bends of a straight boundary would make (sin of the bend below 1e-12 counts as straight)
bool right_turn(const double* x, const double* y, int64_t o, int64_t a, int64_t b) {
    const double c = cross3(x, y, o, a, b);
    if (!(c < 0)) return false;
    const double ax = x[a] - x[o], ay = y[a] - y[o], bx = x[b] - x[o], by = y[b] - y[o];
    return c < -1e-12 * sqrt((ax * ax + ay * ay) * (bx * bx + by * by));
}

// cot of the angle under which chain point m sees (p, q), for m in (p, q), into tmp[m - p - 1]:
// each value is the same IEEE expression as a scalar loop's (no contraction: -ffp-contract=off),
// so the vector widths below only change the speed
__attribute__((always_inline)) inline void cot_scan_body(const double* X, const double* Y, int64_t p, int64_t q,
                                                          double* tmp) {
    const double ax = X[p], ay = Y[p], bx = X[q], by = Y[q];
    const int64_t len = q - p - 1;
    const double* xs = X + p + 1;
    const double* ys = Y + p + 1;
#pragma clang loop vectorize(enable) interleave(enable)
    for (int64_t k = 0; k < len; ++k) {
        const double ux = ax - xs[k], uy = ay - ys[k];
        const double vx = bx - xs[k], vy = by - ys[k];
        const double cr = fabs(ux * vy - uy * vx);
        const double dt = ux * vx + uy * vy;
        const double qt = dt / cr;
        tmp[k] = cr > 0 ? qt : (dt < 0 ? -INFINITY : INFINITY);
    }
}
__attribute__((target("avx2"))) void cot_scan_avx2(const double* X, const double* Y, int64_t p, int64_t q, double* tmp) {
    cot_scan_body(X, Y, p, q, tmp);
}
void cot_scan_base(const double* X, const double* Y, int64_t p, int64_t q, double* tmp) {
    cot_scan_body(X, Y, p, q, tmp);
}

int64_t first_min_base(const double* tmp, int64_t len, double& mn_out) {
    double mn = INFINITY;
    int64_t at = -1;
    for (int64_t k = 0; k < len; ++k)
        if (tmp[k] < mn) {
            mn = tmp[k];
            at = k;
        }
    mn_out = mn;
    return at;
}

// cot_scan + first_min in one pass (AVX-512): the same cot bits per point (the expression above
// with explicit, uncontracted vector operations), each lane keeping its first minimum, the lanes
// merged value first, index second, the tail scalar - the strict '<' scan's pick
__attribute__((target("avx512f,avx512dq"))) int64_t best_avx512(const double* X, const double* Y, int64_t p, int64_t q,
                                                               double& mn_out) {
    const double ax = X[p], ay = Y[p], bx = X[q], by = Y[q];
    const int64_t len = q - p - 1;
    const double* xs = X + p + 1;
    const double* ys = Y + p + 1;
    const __m512d vax = _mm512_set1_pd(ax), vay = _mm512_set1_pd(ay), vbx = _mm512_set1_pd(bx),
                  vby = _mm512_set1_pd(by);
    const __m512d zero = _mm512_setzero_pd(), pinf = _mm512_set1_pd(INFINITY), ninf = _mm512_set1_pd(-INFINITY);
    __m512d mn = pinf;
    __m512i at = _mm512_set1_epi64(-1);
    __m512i idx = _mm512_setr_epi64(0, 1, 2, 3, 4, 5, 6, 7);
    const __m512i eight = _mm512_set1_epi64(8);
    int64_t k = 0;
    for (; k + 8 <= len; k += 8) {
        const __m512d x = _mm512_loadu_pd(xs + k), y = _mm512_loadu_pd(ys + k);
        const __m512d ux = _mm512_sub_pd(vax, x), uy = _mm512_sub_pd(vay, y);
        const __m512d vx = _mm512_sub_pd(vbx, x), vy = _mm512_sub_pd(vby, y);
        const __m512d cr = _mm512_abs_pd(_mm512_sub_pd(_mm512_mul_pd(ux, vy), _mm512_mul_pd(uy, vx)));
        const __m512d dt = _mm512_add_pd(_mm512_mul_pd(ux, vx), _mm512_mul_pd(uy, vy));
        const __m512d qt = _mm512_div_pd(dt, cr);
        // cr > 0 ? qt : (dt < 0 ? -inf : inf)
        const __mmask8 pos = _mm512_cmp_pd_mask(cr, zero, _CMP_GT_OQ);
        const __mmask8 neg = _mm512_cmp_pd_mask(dt, zero, _CMP_LT_OQ);
        const __m512d v = _mm512_mask_mov_pd(_mm512_mask_mov_pd(pinf, neg, ninf), pos, qt);
        const __mmask8 lt = _mm512_cmp_pd_mask(v, mn, _CMP_LT_OQ);
        mn = _mm512_mask_mov_pd(mn, lt, v);
        at = _mm512_mask_mov_epi64(at, lt, idx);
        idx = _mm512_add_epi64(idx, eight);
    }
    alignas(64) double m8[8];
    alignas(64) int64_t a8[8];
    _mm512_store_pd(m8, mn);
    _mm512_store_si512((__m512i*)a8, at);
    double best = INFINITY;
    int64_t pos = -1;
    for (int l = 0; l < 8; ++l)
        if (a8[l] >= 0 && (m8[l] < best || (m8[l] == best && a8[l] < pos))) {
            best = m8[l];
            pos = a8[l];
        }
    for (; k < len; ++k) {
        const double ux = ax - xs[k], uy = ay - ys[k];
        const double vx = bx - xs[k], vy = by - ys[k];
        const double cr = fabs(ux * vy - uy * vx);
        const double dt = ux * vx + uy * vy;
        const double qt = dt / cr;
        const double c = cr > 0 ? qt : (dt < 0 ? -INFINITY : INFINITY);
        if (c < best) {
            best = c;
            pos = k;
        }
    }
    mn_out = best;
    return pos;
}

// the first m in (p, q) with the smallest cot (a strict '<' scan's pick); best_cot receives it
int64_t best_chain_point(const double* X, const double* Y, int64_t p, int64_t q, double* tmp, double& best_cot) {
    static const int isa = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") ? 2
                           : __builtin_cpu_supports("avx2")                                       ? 1
                                                                                                  : 0;
    if (isa == 2) {
        const int64_t at = best_avx512(X, Y, p, q, best_cot);
        return at < 0 ? -1 : p + 1 + at;
    }
    if (isa == 1) cot_scan_avx2(X, Y, p, q, tmp);
    else cot_scan_base(X, Y, p, q, tmp);
    const int64_t len = q - p - 1;
    const int64_t at = first_min_base(tmp, len, best_cot);
    return at < 0 ? -1 : p + 1 + at;
}

struct Key {
    double x, y;
    int64_t i;
};
inline bool key_less(const Key& a, const Key& b) {
    return a.x < b.x || (a.x == b.x && (a.y < b.y || (a.y == b.y && a.i < b.i)));
}
struct Job {
    int64_t p, q;
    int32_t parent;  // pocket triangle on the other side of (p, q), -1 for a hull edge
    int slot;        // which of the parent's nbr slots points back here
};
struct Pocket {
    int64_t p, q;
    int32_t id0;  // its first triangle id
    int err;
    int64_t err_p, err_q;
};
struct Workspace {
    std::vector<Key> keys, keys2;
    std::vector<std::pair<size_t, size_t>> runs, runs2;
    std::vector<char> on_hull;
    std::vector<int64_t> h, hv;
    std::vector<double> X, Y, cot;
    std::vector<Pocket> pockets;
    std::vector<Job> stack;
    std::vector<std::pair<int64_t, int32_t>> chords;
    std::vector<int32_t> next;
};
Workspace& workspace() {
    thread_local Workspace w;
    return w;
}

}  // namespace

using namespace akb;

extern "C" {

int akb_gd_pockets(const double* rx, const double* ry, int nv, int nh, int cap, int32_t* n_out, int32_t* tri,
                   int32_t* nbr, int32_t* edge_tri, int32_t* extra_ptr, int32_t* extra_idx) {
    clear_error();
    AKB_REQUIRE(rx && ry && n_out && tri && nbr && edge_tri && extra_ptr && extra_idx, "null pointer");
    AKB_REQUIRE(nv >= 2 && nh >= 2, "grid of at least 2 x 2 points");
    Ring R{nv, nh, 2 * (int64_t)(nh - 1) + 2 * (int64_t)(nv - 1)};
    const int64_t L = R.L;
    AKB_REQUIRE(cap >= L, "cap >= ring length");
    const int64_t ncells = (int64_t)(nv - 1) * (nh - 1);
    const int64_t base = 2 * ncells;
    AKB_REQUIRE(base + cap < INT32_MAX, "grid too large for 32-bit triangle ids");

    // every buffer below lives in a per-thread workspace: a call runs in a few ms, and fresh
    // allocations of these sizes (mmap'd by malloc) cost it their page faults every time
    Workspace& w = workspace();
    // convex hull of the ring points, collinear points kept (pop on a strict right turn only);
    // sorted as (x, y, index) records (the comparisons read neighbouring memory, not the ring)
    std::vector<Key>& keys = w.keys;
    keys.resize(L);
    for (int64_t i = 0; i < L; ++i) keys[i] = {rx[i], ry[i], i};
    // a lattice's boundary ring is a few monotone runs in this (total) order - four for the C3
    // ring - so a natural merge sort is O(L): strictly descending runs reversed, runs merged in
    // pairs. The order is total (the index breaks ties), so the result is std::sort's exactly.
    {
        auto& runs = w.runs;
        runs.clear();
        for (size_t i = 0; i < (size_t)L && runs.size() <= 64;) {
            size_t j = i + 1;
            if (j < (size_t)L && key_less(keys[j], keys[i])) {
                while (j < (size_t)L && key_less(keys[j], keys[j - 1])) ++j;
                std::reverse(keys.begin() + i, keys.begin() + j);
            } else {
                while (j < (size_t)L && !key_less(keys[j], keys[j - 1])) ++j;
            }
            runs.push_back({i, j});
            i = j;
        }
        if (runs.size() > 64) {
            std::sort(keys.begin(), keys.end(), key_less);
        } else {
            std::vector<Key>& tmp = w.keys2;
            tmp.resize(L);
            while (runs.size() > 1) {  // pairwise merges, ping-pong between the two buffers
                auto& next = w.runs2;
                next.clear();
                for (size_t r = 0; r < runs.size(); r += 2) {
                    if (r + 1 < runs.size()) {
                        std::merge(keys.begin() + runs[r].first, keys.begin() + runs[r].second,
                                   keys.begin() + runs[r + 1].first, keys.begin() + runs[r + 1].second,
                                   tmp.begin() + runs[r].first, key_less);
                        next.push_back({runs[r].first, runs[r + 1].second});
                    } else {
                        std::copy(keys.begin() + runs[r].first, keys.begin() + runs[r].second,
                                  tmp.begin() + runs[r].first);
                        next.push_back(runs[r]);
                    }
                }
                keys.swap(tmp);
                runs.swap(next);
            }
        }
    }
    std::vector<char>& on_hull = w.on_hull;
    on_hull.assign(L, 0);
    for (int pass = 0; pass < 2; ++pass) {
        std::vector<int64_t>& h = w.h;
        h.clear();
        for (int64_t k = 0; k < L; ++k) {
            const int64_t i = pass == 0 ? keys[k].i : keys[L - 1 - k].i;
            while (h.size() >= 2 && right_turn(rx, ry, h[h.size() - 2], h.back(), i)) h.pop_back();
            h.push_back(i);
        }
        for (int64_t i : h) on_hull[i] = 1;
    }
    std::vector<int64_t>& hv = w.hv;
    hv.clear();
    for (int64_t i = 0; i < L; ++i)
        if (on_hull[i]) hv.push_back(i);
    AKB_REQUIRE(hv.size() >= 3, "degenerate point set (all boundary points collinear)");

    for (int64_t e = 0; e < L; ++e) edge_tri[e] = -1;
    // the ring twice over, so a pocket's chain p .. q (q < p + L) is one contiguous index range
    std::vector<double>& X = w.X;
    std::vector<double>& Y = w.Y;
    X.resize(2 * L);
    Y.resize(2 * L);
    for (int64_t i = 0; i < 2 * L; ++i) {
        X[i] = rx[i < L ? i : i - L];
        Y[i] = ry[i < L ? i : i - L];
    }
    // the pockets, one per hull edge that skips ring points. They are independent (disjoint chains
    // and ring edges); triangle ids and chord order are those of one LIFO walk over all of them
    // (the last hull edge's pocket first). One thread walks them in that order (a call is one job of
    // the caller's pool: FaithfulPupil's workers run the runs' calls side by side)
    std::vector<Pocket>& pockets = w.pockets;
    pockets.clear();
    for (size_t k = 0; k < hv.size(); ++k) {
        int64_t p = hv[k], q = hv[(k + 1) % hv.size()];
        if (q <= p) q += L;
        if (q - p < 2) continue;
        // a hull edge that skips a grid corner: the structured triangulation does not apply
        for (int64_t r = p + 1; r < q; ++r)
            if (R.corner(r)) {
                set_error("griddata: the convex hull cuts off a grid corner (ring position %lld); the grid is too "
                          "distorted for the structured triangulation", (long long)(r % L));
                return 2;
            }
        pockets.push_back({p, q, 0, 0, 0, 0});
    }
    int32_t total = 0;
    for (size_t k = pockets.size(); k-- > 0;) {  // the LIFO walk's order: the last pocket first
        pockets[k].id0 = total;
        total += (int32_t)(pockets[k].q - pockets[k].p - 1);  // a pocket of m chain points: m - 2 triangles
    }
    if (total > cap) {
        set_error("griddata: more pocket triangles than cap %d", cap);
        return 2;
    }
    // chords: two per pocket triangle, at 2 (id - id0) within the pocket's block of the list
    std::vector<std::pair<int64_t, int32_t>>& chords = w.chords;
    chords.resize(2 * (size_t)total);
    auto fill = [&](Pocket& P, std::vector<Job>& stack, std::vector<double>& cot) {
        stack.clear();
        stack.push_back({P.p, P.q, -1, -1});
        cot.resize((size_t)(P.q - P.p));
        int32_t n = P.id0;
        while (!stack.empty()) {
            const Job J = stack.back();
            stack.pop_back();
            const int64_t p = J.p, q = J.q;
            // the chain point seeing (p, q) under the largest angle: the first smallest cot = dot / |cross|
            double best_cot = INFINITY;
            const int64_t best = best_chain_point(X.data(), Y.data(), p, q, cot.data(), best_cot);
            if (best < 0 || !(best_cot < INFINITY)) {
                P.err = 1;
                P.err_p = p;
                P.err_q = q;
                return;
            }
            const int64_t m = best;
            const int32_t id = n++;
            const int32_t vp = (int32_t)R.vertex(p), vm = (int32_t)R.vertex(m), vq = (int32_t)R.vertex(q);
            tri[3 * id + 0] = vp;
            tri[3 * id + 1] = vm;
            tri[3 * id + 2] = vq;
            // opposite p: edge (m, q); opposite m: edge (q, p); opposite q: edge (p, m)
            nbr[3 * id + 1] = J.parent < 0 ? -1 : (int32_t)(base + J.parent);
            if (J.parent >= 0) nbr[3 * J.parent + J.slot] = (int32_t)(base + id);
            if (q - m == 1) {
                nbr[3 * id + 0] = -2 - (int32_t)(m % L);
                edge_tri[m % L] = (int32_t)(base + id);
            } else {
                nbr[3 * id + 0] = -1;  // filled by the child
                stack.push_back({m, q, id, 0});
            }
            if (m - p == 1) {
                nbr[3 * id + 2] = -2 - (int32_t)(p % L);
                edge_tri[p % L] = (int32_t)(base + id);
            } else {
                nbr[3 * id + 2] = -1;
                stack.push_back({p, m, id, 2});
            }
            // the base chord (p, q) joins two ring points that are not grid neighbours
            chords[2 * (size_t)id] = {p % L, vq};
            chords[2 * (size_t)id + 1] = {q % L, vp};
        }
    };
    for (auto& P : pockets) fill(P, w.stack, w.cot);
    for (size_t k = pockets.size(); k-- > 0;) {
        const Pocket& P = pockets[k];
        if (P.err) {
            set_error("griddata: degenerate pocket between ring positions %lld and %lld", (long long)P.err_p,
                      (long long)P.err_q);
            return 2;
        }
    }
    const int32_t n = total;
    if ((int64_t)chords.size() > 6 * (int64_t)cap) {
        set_error("griddata: extra-neighbour list overflow");
        return 2;
    }
    // counting sort by ring position, stable: each vertex's chords in the order they were made
    for (int64_t r = 0; r <= L; ++r) extra_ptr[r] = 0;
    for (const auto& c : chords) ++extra_ptr[c.first + 1];
    for (int64_t r = 0; r < L; ++r) extra_ptr[r + 1] += extra_ptr[r];
    std::vector<int32_t>& next = w.next;
    next.assign(extra_ptr, extra_ptr + L);
    for (const auto& c : chords) extra_idx[next[c.first]++] = c.second;
    *n_out = n;
    return 0;
}

}  // extern "C"

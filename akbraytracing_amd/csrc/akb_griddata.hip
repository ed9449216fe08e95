// griddata(points, values, (grid_H, grid_V), method='cubic') of the 'ray_wave' driver on the device
// (AKB_raytrace_20250312.py:3673, :3689).
//
// scipy's cubic griddata is a Clough-Tocher interpolant on the Delaunay triangulation of the
// points (CloughTocher2DInterpolator, scipy 1.15 interpolate/_interpnd): vertex gradients from
// the global curvature-minimising estimate (estimate_gradients_2d_global: each vertex's gradient
// minimises the summed squared second derivative of the edge cubics to its neighbours, solved by
// repeated local 2 x 2 solves), then on each triangle the cubic Bezier patch of the Clough-Tocher
// split, with the cross-boundary derivative taken along the direction to the neighbouring
// triangle's centroid (affine invariant; -1/2 on hull edges), evaluated in extended barycentric
// coordinates. NaN outside the convex hull.
//
// The points are the detector hits of the n_v x n_h ray grid (ray iv * n_h + ih), a smoothly
// deformed lattice, so the Delaunay triangulation is structured: every cell split by the diagonal
// that passes the in-circle test (k_gd_cells) plus the thin "pockets" between the grid's boundary
// ring and its convex hull (akb_gd_pockets, host). k_gd_cells also checks the axis edges are
// locally Delaunay and every cell is convex; a grid that fails is refused, not approximated.
// Gradients: Jacobi sweeps of the same local solve until the largest relative change is below
// tol (scipy runs Gauss-Seidel sweeps to 1e-6; both converge to the same fixed point, the
// iteration matrix contracts by ~1/2 per sweep). Targets: each triangle claims the targets inside
// it (atomicMin of the triangle id: deterministic on shared edges), then each target evaluates
// its triangle's patch.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <mutex>
#include <type_traits>

#include "akb_common.h"
#include "akb_pairwise.h"

namespace akb {
namespace {

struct Grid {
    const double* x;  // (n,) point x (detcenter2[1])
    const double* y;  // (n,) point y (detcenter2[2])
    int nv, nh;
    const uint8_t* diag;  // (nv-1)(nh-1): 0 = split p00-p11, 1 = split p01-p10
    // pockets
    int npock;
    const int32_t* ptri;   // (npock, 3) vertex ids
    const int32_t* pnbr;   // (npock, 3) neighbour opposite vertex k: triangle id, -1 hull, <= -2 ring edge
    const int32_t* edge_tri;  // (L) pocket triangle across ring edge e, -1 (hull edge)
    const int32_t* xptr;   // (L + 1) extra neighbours of ring vertex r (pocket chords)
    const int32_t* xidx;
    // cell rows [row0, row1) the cell pass and the claims visit (a rank's window of a sharded
    // lattice: x, y, diag are then "virtual" global arrays of which only the window's rows, plus
    // two vertex rows below and above, are backed); row1 < 0: every row
    int row0 = 0, row1 = -1;
};

__device__ __forceinline__ int64_t win_cell0(const Grid& g) { return (int64_t)g.row0 * (g.nh - 1); }
__device__ __forceinline__ int64_t win_cell1(const Grid& g) {
    return (int64_t)(g.row1 < 0 ? g.nv - 1 : g.row1) * (g.nh - 1);
}

__device__ __forceinline__ int64_t ncells(const Grid& g) { return (int64_t)(g.nv - 1) * (g.nh - 1); }

__device__ __forceinline__ double orient(double ax, double ay, double bx, double by, double cx, double cy) {
    return (bx - ax) * (cy - ay) - (by - ay) * (cx - ax);
}

// > 0 when d lies inside the circle through a, b, c (any orientation of a, b, c)
__device__ __forceinline__ double incircle(double ax, double ay, double bx, double by, double cx, double cy,
                                           double dx, double dy) {
    const double adx = ax - dx, ady = ay - dy, bdx = bx - dx, bdy = by - dy, cdx = cx - dx, cdy = cy - dy;
    const double A = adx * adx + ady * ady, B = bdx * bdx + bdy * bdy, C = cdx * cdx + cdy * cdy;
    const double det = adx * (bdy * C - B * cdy) - ady * (bdx * C - B * cdx) + A * (bdx * cdy - bdy * cdx);
    const double o = orient(ax, ay, bx, by, cx, cy);
    return o > 0 ? det : -det;
}

// diagonal of cell (iv, ih): 0 (p00-p11) unless p10 lies inside the circle through p00, p01, p11
__device__ int cell_diag(const Grid& g, int iv, int ih, double* viol) {
    const int64_t i00 = (int64_t)iv * g.nh + ih, i01 = i00 + 1, i10 = i00 + g.nh, i11 = i10 + 1;
    const double x0 = g.x[i00], y0 = g.y[i00];
    const double bx = g.x[i01] - x0, by = g.y[i01] - y0;
    const double cx = g.x[i11] - x0, cy = g.y[i11] - y0;
    const double dx = g.x[i10] - x0, dy = g.y[i10] - y0;
    const double ic = incircle(0.0, 0.0, bx, by, cx, cy, dx, dy);
    int d = ic > 0 ? 1 : 0;
    if (viol) {
        // the chosen split must leave two triangles of the same orientation (a convex cell)
        const double s = d == 0 ? orient(0, 0, bx, by, cx, cy) * orient(0, 0, cx, cy, dx, dy)
                                : orient(0, 0, bx, by, dx, dy) * orient(bx, by, cx, cy, dx, dy);
        *viol = s > 0 ? 0.0 : 1.0;
    }
    return d;
}

struct Tri {
    int64_t v[3];
};

// triangle id -> vertices. Cell c = iv * (nh-1) + ih gives ids 2c, 2c + 1:
//   diag 0: (p00, p01, p11), (p00, p11, p10);   diag 1: (p00, p01, p10), (p01, p11, p10)
__device__ __forceinline__ Tri tri_verts(const Grid& g, int64_t t) {
    Tri T;
    const int64_t nc2 = 2 * ncells(g);
    if (t >= nc2) {
        const int64_t j = t - nc2;
        T.v[0] = g.ptri[3 * j];
        T.v[1] = g.ptri[3 * j + 1];
        T.v[2] = g.ptri[3 * j + 2];
        return T;
    }
    const int64_t c = t >> 1;
    const int half = (int)(t & 1);
    const int iv = (int)(c / (g.nh - 1)), ih = (int)(c - (int64_t)iv * (g.nh - 1));
    const int64_t p00 = (int64_t)iv * g.nh + ih, p01 = p00 + 1, p10 = p00 + g.nh, p11 = p10 + 1;
    if (g.diag[c] == 0) {
        if (half == 0) { T.v[0] = p00; T.v[1] = p01; T.v[2] = p11; }
        else { T.v[0] = p00; T.v[1] = p11; T.v[2] = p10; }
    } else {
        if (half == 0) { T.v[0] = p00; T.v[1] = p01; T.v[2] = p10; }
        else { T.v[0] = p01; T.v[1] = p11; T.v[2] = p10; }
    }
    return T;
}

// ring edge index of a cell's boundary side (0 bottom, 1 right, 2 top, 3 left)
__device__ __forceinline__ int64_t ring_edge(const Grid& g, int side, int iv, int ih) {
    const int64_t a = g.nh - 1, b = g.nv - 1;
    switch (side) {
        case 0: return ih;
        case 1: return a + iv;
        case 2: return a + b + (g.nh - 2 - ih);
        default: return 2 * a + b + (g.nv - 2 - iv);
    }
}

// the cell triangle holding ring edge e
__device__ __forceinline__ int64_t ring_edge_tri(const Grid& g, int64_t e) {
    const int64_t a = g.nh - 1, b = g.nv - 1;
    int iv, ih, side;
    if (e < a) { iv = 0; ih = (int)e; side = 0; }
    else if (e < a + b) { iv = (int)(e - a); ih = g.nh - 2; side = 1; }
    else if (e < 2 * a + b) { iv = g.nv - 2; ih = (int)(g.nh - 2 - (e - a - b)); side = 2; }
    else { iv = (int)(g.nv - 2 - (e - 2 * a - b)); ih = 0; side = 3; }
    const int64_t c = (int64_t)iv * (g.nh - 1) + ih;
    const int d = g.diag[c];
    int half;
    if (side == 0) half = 0;
    else if (side == 2) half = 1;
    else if (side == 1) half = d == 0 ? 0 : 1;
    else half = d == 0 ? 1 : 0;
    return 2 * c + half;
}

// neighbour of a cell triangle across its side: another cell's triangle, a pocket, or -1
__device__ __forceinline__ int64_t across_side(const Grid& g, int side, int iv, int ih) {
    if (side == 0) {
        if (iv == 0) return g.edge_tri[ring_edge(g, 0, iv, ih)];
        return 2 * ((int64_t)(iv - 1) * (g.nh - 1) + ih) + 1;  // its top edge: half 1
    }
    if (side == 2) {
        if (iv == g.nv - 2) return g.edge_tri[ring_edge(g, 2, iv, ih)];
        return 2 * ((int64_t)(iv + 1) * (g.nh - 1) + ih);      // its bottom edge: half 0
    }
    if (side == 1) {
        if (ih == g.nh - 2) return g.edge_tri[ring_edge(g, 1, iv, ih)];
        const int64_t c = (int64_t)iv * (g.nh - 1) + ih + 1;      // its left edge
        return 2 * c + (g.diag[c] == 0 ? 1 : 0);
    }
    if (ih == 0) return g.edge_tri[ring_edge(g, 3, iv, ih)];
    const int64_t c = (int64_t)iv * (g.nh - 1) + ih - 1;          // its right edge
    return 2 * c + (g.diag[c] == 0 ? 0 : 1);
}

// neighbour triangle opposite vertex k of triangle t (-1: hull edge)
__device__ int64_t tri_nbr(const Grid& g, int64_t t, int k) {
    const int64_t nc2 = 2 * ncells(g);
    if (t >= nc2) {
        const int32_t v = g.pnbr[3 * (t - nc2) + k];
        if (v >= -1) return v;
        return ring_edge_tri(g, -2 - (int64_t)v);
    }
    const int64_t c = t >> 1;
    const int half = (int)(t & 1);
    const int iv = (int)(c / (g.nh - 1)), ih = (int)(c - (int64_t)iv * (g.nh - 1));
    // side opposite vertex k per (diag, half); -1 = the cell's other triangle
    //   d0 h0 (p00,p01,p11): right, diag, bottom     d0 h1 (p00,p11,p10): top, left, diag
    //   d1 h0 (p00,p01,p10): diag, left, bottom      d1 h1 (p01,p11,p10): top, diag, right
    // packed 3 bits per entry (side + 1), entry index (diag * 2 + half) * 3 + k
    constexpr uint64_t kSide = (2ull << 0) | (0ull << 3) | (1ull << 6) | (3ull << 9) | (4ull << 12) | (0ull << 15) |
                               (0ull << 18) | (4ull << 21) | (1ull << 24) | (3ull << 27) | (0ull << 30) | (2ull << 33);
    const int side = (int)((kSide >> (3 * ((g.diag[c] * 2 + half) * 3 + k))) & 7u) - 1;
    if (side < 0) return 2 * c + (1 - half);
    return across_side(g, side, iv, ih);
}

// ------------------------------------------------------------------ triangulation + checks

// flags: bit 0 a non-convex or degenerate cell, bit 1 an edge that is not locally Delaunay,
// bit 2 a broken pocket adjacency, bits 3 / 4 cells of positive / negative orientation, bit 5 a
// non-finite point
// ------------------------------------------------------------------ targets

constexpr int kClaimAxisLds = 512;  // target axes up to this long go to LDS in the claim kernels

struct Targets {
    const double* gx;  // (mx,) target x axis (grid_H row), ascending
    const double* gy;  // (my,) target y axis (grid_V column), ascending
    int mx, my;
};

// (m - 1) / (a[m-1] - a[0]): the inverse step of a linspace axis (0 for one point)
__device__ __forceinline__ double inv_step(const double* a, int m) {
    const double d = a[m - 1] - a[0];
    return m > 1 && d > 0 ? (m - 1) / d : 0.0;
}

__device__ __forceinline__ int lower_idx(const double* a, int n, double v) {  // first i with a[i] >= v
    int lo = 0, hi = n;
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (a[m] < v) lo = m + 1;
        else hi = m;
    }
    return lo;
}

// barycentric coordinates of (px, py) in triangle T (origin at its last vertex)
__device__ __forceinline__ void bary(const Grid& g, const Tri& T, double px, double py, double (&b)[3]) {
    const double x2 = g.x[T.v[2]], y2 = g.y[T.v[2]];
    const double a00 = g.x[T.v[0]] - x2, a01 = g.x[T.v[1]] - x2;
    const double a10 = g.y[T.v[0]] - y2, a11 = g.y[T.v[1]] - y2;
    const double det = a00 * a11 - a01 * a10;
    const double t00 = a11 / det, t01 = -a01 / det, t10 = -a10 / det, t11 = a00 / det;
    const double dx = px - x2, dy = py - y2;
    b[0] = t00 * dx + t01 * dy;
    b[1] = t10 * dx + t11 * dy;
    b[2] = 1.0 - b[0] - b[1];
}

constexpr double kInsideEps = 100 * 2.220446049250313e-16;

// target index box of triangle T: columns [c0, c1), rows [r0, r1)
__device__ __forceinline__ void tri_box(const Grid& g, const Targets& t, const Tri& T, int& c0, int& c1, int& r0,
                                        int& r1) {
    double xlo = g.x[T.v[0]], xhi = xlo, ylo = g.y[T.v[0]], yhi = ylo;
    for (int k = 1; k < 3; ++k) {
        xlo = fmin(xlo, g.x[T.v[k]]);
        xhi = fmax(xhi, g.x[T.v[k]]);
        ylo = fmin(ylo, g.y[T.v[k]]);
        yhi = fmax(yhi, g.y[T.v[k]]);
    }
    const double padx = (xhi - xlo) * 1e-9, pady = (yhi - ylo) * 1e-9;
    c0 = lower_idx(t.gx, t.mx, xlo - padx);
    c1 = lower_idx(t.gx, t.mx, xhi + padx);
    r0 = lower_idx(t.gy, t.my, ylo - pady);
    r1 = lower_idx(t.gy, t.my, yhi + pady);
}

__device__ __forceinline__ void claim_one(const Grid& g, const Targets& t, const Tri& T, int id, int r, int c,
                                          int* owner) {
    double b[3];
    bary(g, T, t.gx[c], t.gy[r], b);
    if (b[0] >= -kInsideEps && b[1] >= -kInsideEps && b[2] >= -kInsideEps) atomicMin(&owner[(int64_t)r * t.mx + c], id);
}

// candidate index range of the targets of an ascending linspace axis a (m points) in [lo, hi):
// the real-valued indices of lo and hi from the axis's own step, widened by 1e-6 of an index (the
// axis values sit within a few ulp of a0 + c * step); empty when no integer falls between them
__device__ __forceinline__ bool axis_range_at(double a0, int m, double inv_step, double lo, double hi, int& c0,
                                              int& c1) {
    const double e0 = (lo - a0) * inv_step - 1e-6, e1 = (hi - a0) * inv_step + 1e-6;
    if (!(e1 >= 0.0) || !(e0 <= (double)(m - 1))) return false;
    const double f0 = ceil(fmax(e0, 0.0)), f1 = floor(fmin(e1, (double)(m - 1)));
    if (f0 > f1) return false;
    c0 = (int)f0;
    c1 = (int)f1 + 1;
    return true;
}
__device__ __forceinline__ bool axis_range(const double* a, int m, double inv_step, double lo, double hi, int& c0,
                                           int& c1) {
    return axis_range_at(a[0], m, inv_step, lo, hi, c0, c1);
}

// whether axis a (m points, ascending) is a linspace: strictly increasing and every point within
// 1e-6 of an index of a0 + i * step (axis_range's widening); one value per thread of the workgroup
__device__ __forceinline__ bool axis_uniform_part(const double* a, int m, int i) {
    if (i >= m || m < 2) return true;
    const double step = (a[m - 1] - a[0]) / (m - 1);
    if (!(step > 0)) return false;
    if (i > 0 && !(a[i] > a[i - 1])) return false;
    return fabs((a[i] - a[0]) / step - i) <= 1e-7;
}

// the claim kernels' axis test: whether both axes are linspaces (workgroup-wide; every thread)
__device__ __forceinline__ bool axes_uniform(const Targets& t) {
    // the index-box estimate needs evenly spaced axes (np.linspace, the driver's); any other
    // ascending axis takes the exact binary search (lower_idx) of the per-triangle claim
    bool ok = true;
    for (int i = threadIdx.x; i < t.mx || i < t.my; i += blockDim.x)
        ok = ok && axis_uniform_part(t.gx, t.mx, i) && axis_uniform_part(t.gy, t.my, i);
    return __syncthreads_and(ok) != 0;
}

// ---- the claims fused into the cell pass (the cone solve's single-process path, k_gd_cells_strip<true>):
// each cell tests the targets in its own box (rarely any: the 128^2 targets sit ~25 cells apart at C3)
// against its two triangles from the values it holds - claim_cell's box predicate and bary's
// arithmetic on the same values, so the same owners as k_gd_claim_scan + k_gd_claim_hit, with no
// second pass over the lattice
struct TileClaims {
    Targets t;   // the target axes (the device's linspaces, k_gd_axes)
    int* owner;  // (my, mx), INT32_MAX-filled before the pass
};

// ---- the cell pass as wave strips: a wave's 64 lanes hold 64 consecutive vertex columns and walk
// a segment of cell rows upwards (as many rows as puts one wave on every resident slot), a vertex row
// per step (two coalesced loads, issued kStripAhead steps ahead);
// the columns h + 1 and h + 2 come from the lanes above by DPP (wave_shl), a cell's right
// neighbour's diagonal likewise, and the diagonal of the row above is formed one step early - so no
// LDS, no barrier, each vertex loaded once (plus two halo rows per segment) and each diagonal formed
// once. Lanes 0 .. 61 own the cells (lane 62 forms the diagonal lane 61's right edge needs). Every
// test is cell_diag's and the Delaunay checks' arithmetic (the oracle's): the same diagonals and
// flags. With kClaims each cell claims its targets: the candidates from the cell's own box (axis_range
// on linspace axes, else the binary search), then the per-triangle predicate - the same owners.
constexpr int kStripCells = 62, kStripThreads = 256, kStripAhead = 2;

__device__ __forceinline__ int lane_up(int v) {  // lane i gets lane i + 1's value (lane 63: 0, bound_ctrl)
    return __builtin_amdgcn_mov_dpp(v, 0x130, 0xf, 0xf, true);
}
__device__ __forceinline__ double lane_up(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = lane_up((int)(b & 0xffffffffLL)), hi = lane_up((int)(b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

struct StripRow {  // a vertex row at the lane's column h and the two columns after it
    double x, y, x1, y1, x2, y2;
};
__device__ __forceinline__ StripRow strip_row(double x, double y) {
    StripRow r;
    r.x = x;
    r.y = y;
    r.x1 = lane_up(x);
    r.y1 = lane_up(y);
    r.x2 = lane_up(r.x1);
    r.y2 = lane_up(r.y1);
    return r;
}

// the diagonal of the cell between rows a (bottom) and b (top) at the lane's column, and whether
// the split is convex (cell_diag's arithmetic)
__device__ __forceinline__ int strip_diag(const StripRow& a, const StripRow& b, double& viol) {
    const double x0 = a.x, y0 = a.y;
    const double bx = a.x1 - x0, by = a.y1 - y0;
    const double cx = b.x1 - x0, cy = b.y1 - y0;
    const double dx = b.x - x0, dy = b.y - y0;
    const double ic = incircle(0.0, 0.0, bx, by, cx, cy, dx, dy);
    const int d = ic > 0 ? 1 : 0;
    // d = 0: orient(0, b, c) orient(0, c, d); d = 1: orient(0, b, d) orient(b, c, d) - one form with
    // its inputs selected (x - 0.0 is x bit for bit), two orientations a cell instead of four
    const double px = d == 0 ? cx : dx, py = d == 0 ? cy : dy;
    const double ox = d == 0 ? 0.0 : bx, oy = d == 0 ? 0.0 : by;
    const double sgn = (bx * py - by * px) * ((cx - ox) * (dy - oy) - (cy - oy) * (dx - ox));
    viol = sgn > 0 ? 0.0 : 1.0;
    return d;
}

// an edge's local-Delaunay test (the tolerance-scaled in-circle): the edge from (x0, y0) to (cxa, cya), the
// triangle's opposite vertex (mxa, mya), the neighbour's (oxa, oya)
__device__ __forceinline__ bool strip_edge_bad(double x0, double y0, double mxa, double mya, double cxa, double cya,
                                               double oxa, double oya, double tol) {
    const double ax = mxa - x0, ay = mya - y0, cx = cxa - x0, cy = cya - y0;
    const double ox = oxa - x0, oy = oya - y0;
    const double ic = incircle(0.0, 0.0, ax, ay, cx, cy, ox, oy);
    // a non-positive (or NaN) in-circle value never exceeds a non-negative tolerance: the scale only
    // where it can decide (almost never on a Delaunay lattice: its ten FP64 operations a test skipped)
    if (tol >= 0.0 && !(ic > 0.0)) return false;
    const double sc = fmax(fmax(fabs(ax), fabs(ay)), fmax(fmax(fabs(cx), fabs(cy)), fmax(fabs(ox), fabs(oy))));
    return ic > tol * sc * sc * sc * sc;
}

// a cell's claims: its corners (p00, p01, p10, p11) in registers, d its diagonal, c its index
// (ax0, ay0: the axes' first values, read once - a read of the axes here would be a flat load, whose
// wait drains the row loads in flight)
__device__ __forceinline__ void strip_claims(const Targets& t, int* owner, bool uniform, double inv_dx, double inv_dy,
                                             double ax0, double ay0, const double (&vx)[4], const double (&vy)[4], int d,
                                             int64_t c) {
    const double ylo = fmin(fmin(vy[0], vy[1]), fmin(vy[2], vy[3])), yhi = fmax(fmax(vy[0], vy[1]), fmax(vy[2], vy[3]));
    const double pady = (yhi - ylo) * 1e-9;
    int c0, c1, r0, r1;
    bool hit;
    if (uniform) {  // the rows first: a target row meets one cell row in ~25 at C3, so most waves skip the
                    // rest, the x extent included
        hit = axis_range_at(ay0, t.my, inv_dy, ylo - pady, yhi + pady, r0, r1);
        if (hit) {
            const double xlo = fmin(fmin(vx[0], vx[1]), fmin(vx[2], vx[3]));
            const double xhi = fmax(fmax(vx[0], vx[1]), fmax(vx[2], vx[3]));
            const double padx = (xhi - xlo) * 1e-9;
            hit = axis_range_at(ax0, t.mx, inv_dx, xlo - padx, xhi + padx, c0, c1);
        }
    } else {
        const double xlo = fmin(fmin(vx[0], vx[1]), fmin(vx[2], vx[3]));
        const double xhi = fmax(fmax(vx[0], vx[1]), fmax(vx[2], vx[3]));
        const double padx = (xhi - xlo) * 1e-9;
        c0 = lower_idx(t.gx, t.mx, xlo - padx);
        c1 = lower_idx(t.gx, t.mx, xhi + padx);
        r0 = lower_idx(t.gy, t.my, ylo - pady);
        r1 = lower_idx(t.gy, t.my, yhi + pady);
        hit = c0 < c1 && r0 < r1;
    }
    if (!hit) return;
    for (int r = r0; r < r1; ++r) {
        for (int q = c0; q < c1; ++q) {
            const double px = t.gx[q], py = t.gy[r];
#pragma unroll 1
            for (int half = 0; half < 2; ++half) {
                // tri_verts' vertex order, as corner numbers 0 = p00, 1 = p01, 2 = p10, 3 = p11
                int kv[3];
                if (d == 0) {
                    kv[0] = 0;
                    kv[1] = half == 0 ? 1 : 3;
                    kv[2] = half == 0 ? 3 : 2;
                } else {
                    kv[0] = half == 0 ? 0 : 1;
                    kv[1] = half == 0 ? 1 : 3;
                    kv[2] = 2;
                }
                double tx[3], ty[3];
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    tx[k] = kv[k] == 0 ? vx[0] : kv[k] == 1 ? vx[1] : kv[k] == 2 ? vx[2] : vx[3];
                    ty[k] = kv[k] == 0 ? vy[0] : kv[k] == 1 ? vy[1] : kv[k] == 2 ? vy[2] : vy[3];
                }
                double txlo = tx[0], txhi = txlo, tylo = ty[0], tyhi = tylo;
#pragma unroll
                for (int k = 1; k < 3; ++k) {
                    txlo = fmin(txlo, tx[k]);
                    txhi = fmax(txhi, tx[k]);
                    tylo = fmin(tylo, ty[k]);
                    tyhi = fmax(tyhi, ty[k]);
                }
                const double tpx = (txhi - txlo) * 1e-9, tpy = (tyhi - tylo) * 1e-9;
                if (!(px >= txlo - tpx && px < txhi + tpx && py >= tylo - tpy && py < tyhi + tpy)) continue;
                // bary's expressions
                const double x2 = tx[2], y2 = ty[2];
                const double a00 = tx[0] - x2, a01 = tx[1] - x2;
                const double a10 = ty[0] - y2, a11 = ty[1] - y2;
                const double det = a00 * a11 - a01 * a10;
                const double t00 = a11 / det, t01 = -a01 / det, t10 = -a10 / det, t11 = a00 / det;
                const double dx = px - x2, dy = py - y2;
                const double b0 = t00 * dx + t01 * dy, b1 = t10 * dx + t11 * dy, b2 = 1.0 - b0 - b1;
                if (b0 >= -kInsideEps && b1 >= -kInsideEps && b2 >= -kInsideEps)
                    atomicMin(&owner[(int64_t)r * t.mx + q], (int)(2 * c + half));
            }
        }
    }
}

template <bool kClaims = false>
__global__ void __launch_bounds__(kStripThreads) k_gd_cells_strip(Grid g, uint8_t* diag, double tol, unsigned* flags,
                                                                  int seg_rows, TileClaims tc = {}) {
    AKB_CHAIN_PRIORITY();
    const int r_lo = g.row0, r_hi = g.row1 < 0 ? g.nv - 1 : g.row1;  // window cell rows [r_lo, r_hi)
    const int nstrip = (g.nh - 1 + kStripCells - 1) / kStripCells;
    const int nseg = (r_hi - r_lo + seg_rows - 1) / seg_rows;
    const int lane = threadIdx.x & 63;
    const int unit = (int)blockIdx.x * (kStripThreads / 64) + (int)(threadIdx.x >> 6);
    bool uniform = false;
    double inv_dx = 0.0, inv_dy = 0.0, ax0 = 0.0, ay0 = 0.0;
    if constexpr (kClaims) {
        __shared__ double sax[2 * kClaimAxisLds];
        if (tc.t.mx <= kClaimAxisLds && tc.t.my <= kClaimAxisLds) {
            for (int i = threadIdx.x; i < tc.t.mx; i += blockDim.x) sax[i] = tc.t.gx[i];
            for (int i = threadIdx.x; i < tc.t.my; i += blockDim.x) sax[kClaimAxisLds + i] = tc.t.gy[i];
            __syncthreads();
            tc.t.gx = sax;
            tc.t.gy = sax + kClaimAxisLds;
        }
        uniform = axes_uniform(tc.t);
        inv_dx = inv_step(tc.t.gx, tc.t.mx);
        inv_dy = inv_step(tc.t.gy, tc.t.my);
        ax0 = tc.t.gx[0];
        ay0 = tc.t.gy[0];
    }
    if (unit >= nstrip * nseg) return;  // (after the workgroup's barriers)
    const int seg = unit / nstrip, strip = unit - seg * nstrip;
    const int ih = strip * kStripCells + lane, iv0 = r_lo + seg * seg_rows;
    const int iv1 = min(iv0 + seg_rows, r_hi);
    // vertex row r at this lane's column, the index clamped into the lattice and the window's rows + 1
    // (no branch: the wait for a slot then counts only the loads issued after it). Clamped values
    // reach no test: rows past them only feed diagonals that are masked, columns past nh - 1 only
    // right-edge tests that are skipped.
    const int r_top = min(g.nv - 1, r_hi + 1), hc = min(ih, g.nh - 1);
    auto load = [&](int r, double& x, double& y) {
        const int64_t q = (int64_t)min(r, r_top) * g.nh + hc;
        x = g.x[q];
        y = g.y[q];
    };
    // rows iv0 + 2 on in a ring of kStripAhead + 1 register slots (row r in slot (r - iv0) % D), two
    // rows in flight; the step loop unrolled by D = 3, so every slot is a fixed register (a rotation by
    // moves would wait for each load one step after issuing it) and so are the three rows A, B, C
    constexpr int D = kStripAhead + 1;
    double sx[D], sy[D];
#pragma unroll
    for (int k = 2; k < 2 + kStripAhead; ++k) load(iv0 + k, sx[k % D], sy[k % D]);
    double x0, y0, x1, y1;
    load(iv0, x0, y0);
    load(iv0 + 1, x1, y1);
    StripRow A = strip_row(x0, y0), B = strip_row(x1, y1);
    const bool col_cell = ih < g.nh - 1;                   // a cell at this column
    const bool own_lane = lane < kStripCells && col_cell;  // (lanes 62 and 63 own none)
    double bad = 0.0;
    int d = col_cell ? strip_diag(A, B, bad) : 0;
    unsigned acc = 0;
    for (int j0 = 0; j0 < iv1 - iv0; j0 += D) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
            const int iv = iv0 + j0 + u;
            if (iv >= iv1) break;
            // row iv + 2 arrived (issued kStripAhead steps ago); row iv + 2 + kStripAhead issued now
            const StripRow C = strip_row(sx[(u + 2) % D], sy[(u + 2) % D]);
            load(iv + 2 + kStripAhead, sx[(u + 2 + kStripAhead) % D], sy[(u + 2 + kStripAhead) % D]);
            // the row above's diagonal (this lane's next step) and the right neighbour's on this row
            const int jv = iv + 1;
            double bad_up = 0.0;
            const int dup = (col_cell && jv < g.nv - 1 && jv <= r_hi) ? strip_diag(B, C, bad_up) : 0;
            const int dn = lane_up(d);
            if (own_lane) {
                const int64_t c = (int64_t)iv * (g.nh - 1) + ih;
                diag[c] = (uint8_t)d;
                unsigned f = bad > 0 ? 1u : 0u;
                if (!isfinite(A.x) || !isfinite(A.y)) f |= 32u;
                {
                    const double o = orient(A.x, A.y, A.x1, A.y1, B.x1, B.y1);
                    f |= o > 0 ? 8u : (o < 0 ? 16u : 1u);
                }
                if (ih + 1 < g.nh - 1) {  // right edge p01-p11 against the next cell's left triangle
                    const double mx = d == 0 ? A.x : B.x, my = d == 0 ? A.y : B.y;
                    const double ox = dn == 0 ? B.x2 : A.x2, oy = dn == 0 ? B.y2 : A.y2;
                    if (strip_edge_bad(A.x1, A.y1, mx, my, B.x1, B.y1, ox, oy, tol)) f |= 2u;
                }
                if (iv + 1 < g.nv - 1) {  // top edge p10-p11 against the next row's bottom triangle
                    const double mx = d == 0 ? A.x : A.x1, my = d == 0 ? A.y : A.y1;
                    const double ox = dup == 0 ? C.x1 : C.x, oy = dup == 0 ? C.y1 : C.y;
                    if (strip_edge_bad(B.x, B.y, mx, my, B.x1, B.y1, ox, oy, tol)) f |= 2u;
                }
                acc |= f;
                if constexpr (kClaims) {
                    const double vx[4] = {A.x, A.x1, B.x, B.x1}, vy[4] = {A.y, A.y1, B.y, B.y1};
                    strip_claims(tc.t, tc.owner, uniform, inv_dx, inv_dy, ax0, ay0, vx, vy, d, c);
                }
            }
            A = B;
            B = C;
            d = dup;
            bad = bad_up;
        }
    }
    for (int off = 32; off > 0; off >>= 1) acc |= __shfl_down(acc, off);
    if (lane == 0) {
        const unsigned cur = __hip_atomic_load(flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((cur | acc) != cur) atomicOr(flags, acc);
    }
}

// ring positions -> coordinates, for the host pocket builder (bit 5 of flags: a non-finite one)
__global__ void k_gd_ring(Grid g, double* rx, double* ry, unsigned* flags) {
    AKB_CHAIN_PRIORITY();
    const int64_t a = g.nh - 1, b = g.nv - 1, L = 2 * a + 2 * b;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < L; r += (int64_t)gridDim.x * blockDim.x) {
        int64_t v;
        if (r < a) v = r;
        else if (r < a + b) v = (r - a) * g.nh + (g.nh - 1);
        else if (r < 2 * a + b) v = (int64_t)(g.nv - 1) * g.nh + (g.nh - 1 - (r - a - b));
        else v = (int64_t)(g.nv - 1 - (r - 2 * a - b)) * g.nh;
        rx[r] = g.x[v];
        ry[r] = g.y[v];
        if (!isfinite(rx[r]) || !isfinite(ry[r])) atomicOr(flags, 32u);
    }
}

// the pockets against the triangles they border: every pocket edge locally Delaunay (bit 1)
__global__ void k_gd_check_pockets(Grid g, double tol, unsigned* flags) {
    AKB_CHAIN_PRIORITY();
    const int64_t nc2 = 2 * ncells(g);
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < g.npock; j += (int64_t)gridDim.x * blockDim.x) {
        const Tri T = tri_verts(g, nc2 + j);
        for (int k = 0; k < 3; ++k) {
            const int64_t n = tri_nbr(g, nc2 + j, k);
            if (n < 0) continue;
            const Tri N = tri_verts(g, n);
            // the neighbour's vertex that is not on the shared edge
            int64_t o = -1;
            for (int q = 0; q < 3; ++q)
                if (N.v[q] != T.v[(k + 1) % 3] && N.v[q] != T.v[(k + 2) % 3]) o = N.v[q];
            if (o < 0) {
                atomicOr(flags, 4u);
                continue;
            }
            const double x0 = g.x[T.v[0]], y0 = g.y[T.v[0]];
            const double bx = g.x[T.v[1]] - x0, by = g.y[T.v[1]] - y0, cx = g.x[T.v[2]] - x0, cy = g.y[T.v[2]] - y0;
            const double ox = g.x[o] - x0, oy = g.y[o] - y0;
            const double s = fmax(fmax(fabs(bx), fabs(by)), fmax(fmax(fabs(cx), fabs(cy)), fmax(fabs(ox), fabs(oy))));
            if (incircle(0.0, 0.0, bx, by, cx, cy, ox, oy) > tol * s * s * s * s) atomicOr(flags, 2u);
        }
    }
}

// ------------------------------------------------------------------ gradients
//
// scipy's local solve at vertex i (estimate_gradients_2d_global, scipy 1.15 interpolate/_interpnd):
// over the edges e = p_j - p_i, with r3 = |e|^-3,
//     Q = 4 sum r3 e e^T,    s = sum (6 (f_i - f_j) + 2 e.g_j) r3 e,    g_i <- -Q^-1 s.
// With M = r3 e e^T and w = r3 e per edge this is g_i <- c - P S: c = -Q^-1 sum 6 (f_i - f_j) w and
// P = 2 Q^-1 depend on the geometry and the values only, S = sum M g_j on the iterate. Every kernel
// below forms them in one arithmetic (edge_geom, acc_edge, vertex_consts, jacobi_y) and one edge
// order - left, right, down, up, then the diagonals present (those of cells (iv-1, ih-1), (iv-1, ih),
// (iv, ih-1), (iv, ih)); a ring vertex's pocket chords are summed over lanes and added to those -
// so any two kernels reach the same iterate bit for bit. A kernel that keeps the geometry (the cone
// patches) then spends four FMAs per edge and sweep. An edge's M and w are the same from both of
// its ends (the edge vector only changes sign), and an absent edge taken as M = 0 adds exact zeros
// (S starts at +0 and a zero product never turns it negative), so the patches may run all eight
// slots without branches and still give the gather kernels' bits.

__device__ __forceinline__ int64_t ring_pos(const Grid& g, int iv, int ih) {
    const int64_t a = g.nh - 1, b = g.nv - 1;
    if (iv == 0) return ih;
    if (ih == g.nh - 1) return a + iv;
    if (iv == g.nv - 1) return a + b + (g.nh - 1 - ih);
    if (ih == 0) return 2 * a + b + (g.nv - 1 - iv);
    return -1;
}

// ring vertex r's lattice index (the ring in k_gd_ring's order)
__device__ __forceinline__ int64_t ring_vertex(const Grid& g, int64_t r) {
    const int64_t ra = g.nh - 1, rb = g.nv - 1;
    if (r < ra) return r;
    if (r < ra + rb) return (r - ra) * g.nh + (g.nh - 1);
    if (r < 2 * ra + rb) return (int64_t)(g.nv - 1) * g.nh + (g.nh - 1 - (r - ra - rb));
    return (int64_t)(g.nv - 1 - (r - 2 * ra - rb)) * g.nh;
}

// one edge's geometry: M = r3 e e^T (mxx, mxy, myy) and w = r3 e. r3 from the hardware reciprocal
// square root and one Newton step (relative error ~1e-16; the solve is an iteration, not
// reproduced from scipy bit for bit)
struct EdgeG {
    double mxx, mxy, myy, wx, wy;
};

__device__ __forceinline__ EdgeG edge_geom(double ex, double ey) {
    const double l2 = ex * ex + ey * ey;
    double r = __builtin_amdgcn_rsq(l2);
    r = r * __builtin_fma(-0.5 * l2 * r, r, 1.5);
    const double r3 = r * r * r;
    EdgeG e;
    e.wx = ex * r3;
    e.wy = ey * r3;
    e.mxx = ex * e.wx;
    e.mxy = ex * e.wy;
    e.myy = ey * e.wy;
    return e;
}

// a vertex's sums: Q / 4 (geometry, shared by the value sets), c-sums and S per value set. S runs
// as two chains - the axis edges (and chords) in s, the diagonals in d - folded s + d before use
// (acc_fold), which halves the dependent FMA chain of a patch sweep
template <int NV>
struct GradAcc {
    double q0 = 0, q1 = 0, q3 = 0;
    double c0[NV] = {}, c1[NV] = {};
    double s0[NV] = {}, s1[NV] = {};
    double d0[NV] = {}, d1[NV] = {};
};

constexpr int kAccWords(int nv) { return 3 + 4 * nv; }  // a GradAcc in ring_acc / chord buffers

template <int NV, bool kDiag = false>
__device__ __forceinline__ void acc_edge(GradAcc<NV>& A, const EdgeG& e, const double (&fi)[NV], const double (&fj)[NV],
                                         const double (&gxj)[NV], const double (&gyj)[NV]) {
    A.q0 = A.q0 + e.mxx;
    A.q1 = A.q1 + e.mxy;
    A.q3 = A.q3 + e.myy;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const double c6 = 6 * (fi[v] - fj[v]);
        A.c0[v] = __builtin_fma(c6, e.wx, A.c0[v]);
        A.c1[v] = __builtin_fma(c6, e.wy, A.c1[v]);
        double& t0 = kDiag ? A.d0[v] : A.s0[v];
        double& t1 = kDiag ? A.d1[v] : A.s1[v];
        t0 = __builtin_fma(e.mxy, gyj[v], __builtin_fma(e.mxx, gxj[v], t0));
        t1 = __builtin_fma(e.myy, gyj[v], __builtin_fma(e.mxy, gxj[v], t1));
    }
}

// S = axis chain + diagonal chain (d = 0 after: the sums are then ready to add, store or solve)
template <int NV>
__device__ __forceinline__ GradAcc<NV>& acc_fold(GradAcc<NV>& A) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        A.s0[v] = A.s0[v] + A.d0[v];
        A.s1[v] = A.s1[v] + A.d1[v];
        A.d0[v] = A.d1[v] = 0.0;
    }
    return A;
}

// A = A + B, every word (chords + lattice edges)
template <int NV>
__device__ __forceinline__ void acc_add(GradAcc<NV>& A, const GradAcc<NV>& B) {
    A.q0 = A.q0 + B.q0;
    A.q1 = A.q1 + B.q1;
    A.q3 = A.q3 + B.q3;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        A.c0[v] = A.c0[v] + B.c0[v];
        A.c1[v] = A.c1[v] + B.c1[v];
        A.s0[v] = A.s0[v] + B.s0[v];
        A.s1[v] = A.s1[v] + B.s1[v];
    }
}

// the fixed butterfly over W lanes (a lane group's chord sums; zero partners change no bits)
template <int NV, int W>
__device__ __forceinline__ void acc_reduce(GradAcc<NV>& A) {
    for (int off = W / 2; off > 0; off >>= 1) {
        A.q0 += __shfl_down(A.q0, off, W);
        A.q1 += __shfl_down(A.q1, off, W);
        A.q3 += __shfl_down(A.q3, off, W);
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            A.c0[v] += __shfl_down(A.c0[v], off, W);
            A.c1[v] += __shfl_down(A.c1[v], off, W);
            A.s0[v] += __shfl_down(A.s0[v], off, W);
            A.s1[v] += __shfl_down(A.s1[v], off, W);
        }
    }
}

template <int NV>
__device__ __forceinline__ void acc_store(double* d, const GradAcc<NV>& A) {
    d[0] = A.q0;
    d[1] = A.q1;
    d[2] = A.q3;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        d[3 + 4 * v] = A.c0[v];
        d[4 + 4 * v] = A.c1[v];
        d[5 + 4 * v] = A.s0[v];
        d[6 + 4 * v] = A.s1[v];
    }
}

template <int NV>
__device__ __forceinline__ GradAcc<NV> acc_load(const double* d) {
    GradAcc<NV> A;
    A.q0 = d[0];
    A.q1 = d[1];
    A.q3 = d[2];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        A.c0[v] = d[3 + 4 * v];
        A.c1[v] = d[4 + 4 * v];
        A.s0[v] = d[5 + 4 * v];
        A.s1[v] = d[6 + 4 * v];
    }
    return A;
}

// the vertex's constants of value set v: c = -Q^-1 csum, P = 2 Q^-1 (symmetric)
struct VConst {
    double c0, c1, p00, p01, p11;
};

template <int NV>
__device__ __forceinline__ VConst vertex_consts(const GradAcc<NV>& A, int v) {
    const double q0 = 4 * A.q0, q1 = 4 * A.q1, q3 = 4 * A.q3;
    const double inv = 1.0 / (q0 * q3 - q1 * q1);
    VConst k;
    k.c0 = -((q3 * A.c0[v] - q1 * A.c1[v]) * inv);
    k.c1 = -((q0 * A.c1[v] - q1 * A.c0[v]) * inv);
    const double i2 = 2 * inv;
    k.p00 = q3 * i2;
    k.p01 = -(q1 * i2);
    k.p11 = q0 * i2;
    return k;
}

// the Jacobi step's new gradient y = c - P S
__device__ __forceinline__ void jacobi_y(const VConst& k, double s0, double s1, double& y0, double& y1) {
    y0 = k.c0 - __builtin_fma(k.p01, s1, k.p00 * s0);
    y1 = k.c1 - __builtin_fma(k.p01, s0, k.p11 * s1);
}

// scipy's change measure of a Jacobi step from (gx, gy) to y (its stopping rule's quantity)
__device__ __forceinline__ double change_of(double gx, double gy, double y0, double y1) {
    return fmax(fabs(gx - y0), fabs(gy - y1)) / fmax(1.0, fmax(fabs(y0), fabs(y1)));
}

// sweep j's weight and predecessor form: mode 0 plain (y itself), 2 against the predecessor p
// (omega (y - p) + p), 1 the same against a zero predecessor (the caller passes p = 0)
struct ConeStep {
    int mode;
    double omega;
};

__device__ __forceinline__ double cheb(const ConeStep& st, double y, double p) {
    return st.mode == 0 ? y : __builtin_fma(st.omega, y - p, p);  // mode 1: p = 0
}

// Chebyshev semi-iteration for a Jacobi spectrum in [-1/2, 1/2] (the local problem is block
// diagonally dominant by a factor 2): ~0.27 error contraction per sweep instead of
// Jacobi's 1/2. The global kernels' form of ConeStep: gprev = x_{k-1} (mode 2), zero_prev (mode 1).
struct Cheb {
    const double* gprev;
    double omega;
    int zero_prev = 0;
};

// the solve of value set v at output offset o (gin nullptr: x_k = 0); returns the change measure
template <int NV>
__device__ __forceinline__ double grad_solve(const GradAcc<NV>& A, int v, const double* gin, double* gout, int64_t o,
                                             const Cheb& ch) {
    const VConst k = vertex_consts<NV>(A, v);
    double y0, y1;
    jacobi_y(k, A.s0[v], A.s1[v], y0, y1);  // A folded by the caller
    const double gx = gin ? gin[o] : 0.0, gy = gin ? gin[o + 1] : 0.0;
    const ConeStep st{ch.gprev ? 2 : (ch.zero_prev ? 1 : 0), ch.omega};
    const double px = ch.gprev ? ch.gprev[o] : 0.0, py = ch.gprev ? ch.gprev[o + 1] : 0.0;
    gout[o] = cheb(st, y0, px);
    gout[o + 1] = cheb(st, y1, py);
    return change_of(gx, gy, y0, y1);
}

// one edge i -> j read from global memory (gin nullptr: x = 0)
template <int NV>
__device__ __forceinline__ void grad_edge(const Grid& g, int64_t n, int64_t j, double xi, double yi,
                                          const double (&fi)[NV], const double* __restrict__ f,
                                          const double* __restrict__ gin, GradAcc<NV>& A) {
    double fj[NV], gxj[NV], gyj[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        fj[v] = f[v * n + j];
        gxj[v] = gin ? gin[2 * (v * n + j)] : 0.0;
        gyj[v] = gin ? gin[2 * (v * n + j) + 1] : 0.0;
    }
    acc_edge<NV>(A, edge_geom(g.x[j] - xi, g.y[j] - yi), fi, fj, gxj, gyj);
}

// ring vertex r's pocket chords over a group of W lanes (sub: the lane in the group), reduced by the
// group's butterfly (zeros from the lanes past the chord list)
template <int NV, int W, int kB = 4>
__device__ __forceinline__ GradAcc<NV> chord_sums(const Grid& g, int64_t n, int64_t r, int sub, double xi, double yi,
                                                  const double (&fi)[NV], const double* __restrict__ f,
                                                  const double* __restrict__ gin) {
    GradAcc<NV> A;
    // kB of the lane's chords at a time: their indices, then their data, loaded before the first
    // edge sum (the same edges in the same order; a loop of index-load, data-load, sum waited out
    // two memory latencies per chord)
    const int32_t k1 = g.xptr[r + 1];
    for (int32_t k0 = g.xptr[r] + sub; k0 < k1; k0 += kB * W) {
        int64_t js[kB];
#pragma unroll
        for (int b = 0; b < kB; ++b) js[b] = k0 + b * W < k1 ? g.xidx[k0 + b * W] : -1;
        double xj[kB], yj[kB], fj[kB][NV], gxj[kB][NV], gyj[kB][NV];
#pragma unroll
        for (int b = 0; b < kB; ++b) {
            const int64_t j = js[b] < 0 ? 0 : js[b];
            xj[b] = g.x[j];
            yj[b] = g.y[j];
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                fj[b][v] = f[v * n + j];
                gxj[b][v] = gin ? gin[2 * (v * n + j)] : 0.0;
                gyj[b][v] = gin ? gin[2 * (v * n + j) + 1] : 0.0;
            }
        }
#pragma unroll
        for (int b = 0; b < kB; ++b)
            if (js[b] >= 0) acc_edge<NV>(A, edge_geom(xj[b] - xi, yj[b] - yi), fi, fj[b], gxj[b], gyj[b]);
    }
    acc_reduce<NV, W>(A);  // (the chords run in the axis chain: d stays 0)
    return A;
}

template <int W>
__device__ __forceinline__ void change_max_n(double worst, unsigned long long* chg) {
    __shared__ double red[W / 64];
    for (int off = 32; off > 0; off >>= 1) worst = fmax(worst, __shfl_down(worst, off));
    if (W > 64) {
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = worst;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        for (int w = 1; w < W / 64; ++w) worst = fmax(worst, red[w]);
        const unsigned long long bits = (unsigned long long)__double_as_longlong(worst);
        if (chg && worst > 0 && __hip_atomic_load(chg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < bits)
            atomicMax(chg, bits);
    }
}

// ring vertices after k_gd_sweeps' second sweep: one wave each adds the pocket chords of gin to
// the lattice-edge sums the sweep kernel left in ring_acc, then solves
template <int NV>
__global__ void __launch_bounds__(kBlock) k_gd_grad_ring(Grid g, const double* __restrict__ f,
                                                         const double* __restrict__ gin, double* __restrict__ gout,
                                                         const double* __restrict__ ring_acc, unsigned long long* chg,
                                                         Cheb ch) {
    const int64_t n = (int64_t)g.nv * g.nh;
    const int64_t L = 2 * (int64_t)(g.nh - 1) + 2 * (int64_t)(g.nv - 1);
    const int lane = threadIdx.x & 63;
    double worst = 0.0;
    for (int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; r < L;
         r += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        const int64_t i = ring_vertex(g, r);
        const double xi = g.x[i], yi = g.y[i];
        double fi[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) fi[v] = f[v * n + i];
        GradAcc<NV> A = chord_sums<NV, 64>(g, n, r, lane, xi, yi, fi, f, gin);
        if (lane == 0) {
            acc_add<NV>(A, acc_load<NV>(ring_acc + r * kAccWords(NV)));
#pragma unroll
            for (int v = 0; v < NV; ++v) worst = fmax(worst, grad_solve<NV>(A, v, gin, gout, 2 * (v * n + i), ch));
        }
    }
    change_max_n<kBlock>(worst, chg);
}

// pocket-chord sums of every ring vertex from gradients gin (nullptr = zeros), one wave each
template <int NV>
__global__ void __launch_bounds__(kBlock) k_gd_ring_chords(Grid g, const double* __restrict__ f,
                                                           const double* __restrict__ gin, double* __restrict__ out) {
    const int64_t n = (int64_t)g.nv * g.nh;
    const int64_t L = 2 * (int64_t)(g.nh - 1) + 2 * (int64_t)(g.nv - 1);
    const int lane = threadIdx.x & 63;
    for (int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; r < L;
         r += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        const int64_t i = ring_vertex(g, r);
        const double xi = g.x[i], yi = g.y[i];
        double fi[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) fi[v] = f[v * n + i];
        const GradAcc<NV> A = chord_sums<NV, 64>(g, n, r, lane, xi, yi, fi, f, gin);
        if (lane == 0) acc_store<NV>(out + r * kAccWords(NV), A);
    }
}

// ------------------------------------------------------------------ register sweeps (two per launch)
//
// k_gd_sweeps: each wave owns a strip of columns (one lane per column, the two outer lanes on each
// side are halo) and walks down a chunk of rows; the rows it works on sit in registers and the
// left / right neighbours come from the adjacent lanes (DPP wave shifts), so there is no LDS and
// no barrier. kK = 2 does two Chebyshev sweeps per launch, the second one row behind the first
// (wavefront temporal blocking): the first sweep's values are formed one column and one row into
// the halo so the second has its neighbours, and only x, y, f and the two gradient sets of the
// rows are read from HBM once per two sweeps. Ring vertices take their pocket chords from
// k_gd_ring_chords (x_k, before the launch); in the second sweep they only store their grid-edge
// sums and k_gd_grad_ring adds the chords of x_{k+1} and solves after the launch.

// lane l gets lane l - 1's value (DPP wave_shr:1) / lane l + 1's (wave_shl:1); doubles: one
// v_mov_b32_dpp per half with bound_ctrl (lane 0 / lane 63 read 0: halo lanes). (The cell flags are
// loaded per lane rather than shifted: an int shifted this way read the neighbour on the wrong side
// at a flag change on the MI355X.)
__device__ __forceinline__ double lane_prev(double v) {
    return __hiloint2double(__builtin_amdgcn_mov_dpp(__double2hiint(v), 0x138, 0xf, 0xf, true),
                            __builtin_amdgcn_mov_dpp(__double2loint(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ double lane_next(double v) {
    return __hiloint2double(__builtin_amdgcn_mov_dpp(__double2hiint(v), 0x130, 0xf, 0xf, true),
                            __builtin_amdgcn_mov_dpp(__double2loint(v), 0x130, 0xf, 0xf, true));
}

template <int NV>
struct RV {  // one vertex of a row: position, values, gradients, diagonal flags of cells (row, col), (row, col - 1)
    double x, y, f[NV], gx[NV], gy[NV];
    int d, dl;
};

template <int NV, bool kNext>
__device__ __forceinline__ RV<NV> rv_shift(const RV<NV>& r) {
    RV<NV> o;
    o.x = kNext ? lane_next(r.x) : lane_prev(r.x);
    o.y = kNext ? lane_next(r.y) : lane_prev(r.y);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        o.f[v] = kNext ? lane_next(r.f[v]) : lane_prev(r.f[v]);
        o.gx[v] = kNext ? lane_next(r.gx[v]) : lane_prev(r.gx[v]);
        o.gy[v] = kNext ? lane_next(r.gy[v]) : lane_prev(r.gy[v]);
    }
    o.d = o.dl = 0;  // the flags are loaded per lane (RV::dl), never shifted
    return o;
}

template <int NV, bool kDiag>
__device__ __forceinline__ void edge_rv(const RV<NV>& o, const RV<NV>& c, GradAcc<NV>& A) {
    acc_edge<NV, kDiag>(A, edge_geom(o.x - c.x, o.y - c.y), c.f, o.f, o.gx, o.gy);
}

// the lattice-edge sums of the vertex in row `cur` (wave-uniform control flow: the lane shifts run
// in every lane; only the shifts some lane of the wave needs are made)
template <int NV>
__device__ __forceinline__ GradAcc<NV> vertex_sums(const RV<NV>& up, const RV<NV>& cur, const RV<NV>& dn,
                                                   bool hl, bool hr, bool hu, bool hd) {
    const bool ul = hu && hl && up.dl == 0, ur = hu && hr && up.d == 1;
    const bool dl = hd && hl && cur.dl == 1, dr = hd && hr && cur.d == 0;
    GradAcc<NV> A;
    {
        const RV<NV> L = rv_shift<NV, false>(cur);
        if (hl) edge_rv<NV, false>(L, cur, A);
    }
    {
        const RV<NV> R = rv_shift<NV, true>(cur);
        if (hr) edge_rv<NV, false>(R, cur, A);
    }
    if (hu) edge_rv<NV, false>(up, cur, A);
    if (hd) edge_rv<NV, false>(dn, cur, A);
    if (__any(ul)) {
        const RV<NV> N = rv_shift<NV, false>(up);
        if (ul) edge_rv<NV, true>(N, cur, A);
    }
    if (__any(ur)) {
        const RV<NV> N = rv_shift<NV, true>(up);
        if (ur) edge_rv<NV, true>(N, cur, A);
    }
    if (__any(dl)) {
        const RV<NV> N = rv_shift<NV, false>(dn);
        if (dl) edge_rv<NV, true>(N, cur, A);
    }
    if (__any(dr)) {
        const RV<NV> N = rv_shift<NV, true>(dn);
        if (dr) edge_rv<NV, true>(N, cur, A);
    }
    return acc_fold<NV>(A);
}

template <int NV>
struct SweepArgs {
    const double* f;       // (NV, n) values
    const double* gin;     // (NV, n, 2) x_k, nullptr = zeros
    const double* gprev;   // (NV, n, 2) x_{k-1} for the first sweep's Chebyshev step, nullptr = plain
    double om1, om2;       // the two sweeps' weights
    double* gout1;         // x_{k+1}
    double* gout2;         // x_{k+2} (kK = 2)
    const double* chords;  // (L, kAccWords) pocket-chord sums of x_k (k_gd_ring_chords)
    double* ring_acc;      // (L, kAccWords) grid-edge sums of x_{k+1} at ring vertices (kK = 2)
    unsigned long long* chg;  // [2]: largest relative change of each sweep
    int rows;              // rows per wave
};

template <int NV, int kK, int kWaves>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kWaves)))
k_gd_sweeps(Grid g, SweepArgs<NV> a) {
    constexpr int kHalo = kK;             // halo lanes on each side
    constexpr int kOwn = 64 - 2 * kHalo;  // columns a wave owns
    const int64_t n = (int64_t)g.nv * g.nh;
    const int lane = threadIdx.x & 63;
    const int wave = (int)((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6);
    const int nstrips = (g.nh + kOwn - 1) / kOwn;
    const int nchunks = (g.nv + a.rows - 1) / a.rows;
    double worst1 = 0.0, worst2 = 0.0;
    if (wave < nstrips * nchunks) {
        const int strip = wave % nstrips, chunk = wave / nstrips;
        const int ih = strip * kOwn + lane - kHalo;
        const bool col = ih >= 0 && ih < g.nh;
        const bool own = col && lane >= kHalo && lane < 64 - kHalo;
        const int r0 = chunk * a.rows, r1 = min(r0 + a.rows, g.nv);
        const bool hl = ih > 0, hr = ih < g.nh - 1;
        // geometry (x, y, f, d) and x_k of row rr; x_{k-1} of row rr
        auto load = [&](int rr, RV<NV>& r) {
            r.x = r.y = 0.0;
            r.d = r.dl = 0;
#pragma unroll
            for (int v = 0; v < NV; ++v) r.f[v] = r.gx[v] = r.gy[v] = 0.0;
            if (!col || rr < 0 || rr >= g.nv) return;
            const int64_t i = (int64_t)rr * g.nh + ih;
            r.x = g.x[i];
            r.y = g.y[i];
            const int64_t c = (int64_t)rr * (g.nh - 1) + ih;
            r.d = (rr < g.nv - 1 && ih < g.nh - 1) ? g.diag[c] : 0;
            r.dl = (rr < g.nv - 1 && ih > 0) ? g.diag[c - 1] : 0;
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                r.f[v] = a.f[v * n + i];
                if (a.gin) {
                    r.gx[v] = a.gin[2 * (v * n + i)];
                    r.gy[v] = a.gin[2 * (v * n + i) + 1];
                }
            }
        };
        auto load_prev = [&](int rr, double (&px)[NV], double (&py)[NV]) {
#pragma unroll
            for (int v = 0; v < NV; ++v) px[v] = py[v] = 0.0;
            if (!a.gprev || !col || rr < 0 || rr >= g.nv) return;
            const int64_t i = (int64_t)rr * g.nh + ih;
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                px[v] = a.gprev[2 * (v * n + i)];
                py[v] = a.gprev[2 * (v * n + i) + 1];
            }
        };
        const ConeStep st1{a.gprev ? 2 : 0, a.om1}, st2{2, a.om2};
        // sweep 1 of row i (rows up / cur / dn) -> s (x_{k+1} of row i, NV x 2)
        auto sweep1 = [&](int i, const RV<NV>& up, const RV<NV>& cur, const RV<NV>& dn, const double (&px)[NV],
                          const double (&py)[NV], RV<NV>& s) {
            s = cur;  // geometry and values carry over; gradients replaced below
            GradAcc<NV> A = vertex_sums<NV>(up, cur, dn, hl, hr, i > 0, i < g.nv - 1);
            if (!col || i < 0 || i >= g.nv) return;
            const int64_t r = ring_pos(g, i, ih);
            if (r >= 0) {  // pocket chords of x_k, then the lattice edges
                GradAcc<NV> C = acc_load<NV>(a.chords + r * kAccWords(NV));
                acc_add<NV>(C, A);
                A = C;
            }
            const bool mine = own && i >= r0 && i < r1;
            const int64_t o = (int64_t)i * g.nh + ih;
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const VConst k = vertex_consts<NV>(A, v);
                double y0, y1;
                jacobi_y(k, A.s0[v], A.s1[v], y0, y1);
                const double ox = cheb(st1, y0, px[v]), oy = cheb(st1, y1, py[v]);
                s.gx[v] = ox;
                s.gy[v] = oy;
                if (mine) {
                    worst1 = fmax(worst1, change_of(cur.gx[v], cur.gy[v], y0, y1));
                    a.gout1[2 * (v * n + o)] = ox;
                    a.gout1[2 * (v * n + o) + 1] = oy;
                }
            }
        };
        RV<NV> G0, G1, G2, G3;  // x_k rows i - 2 .. i + 1 (kK = 2) / i - 1 .. i + 1 (kK = 1: G1 .. G3)
        RV<NV> S0, S1, S2;      // x_{k+1} rows i - 2 .. i
        double px[NV], py[NV], qx[NV], qy[NV];
        const int first = kK == 2 ? r0 - 1 : r0;  // rows of sweep 1
        const int last = kK == 2 ? r1 : r1 - 1;
        load(first - 2, G0);
        load(first - 1, G1);
        load(first, G2);
        load(first + 1, G3);
        load_prev(first, px, py);
        S0 = G0;
        S1 = G1;
        for (int i = first; i <= last; ++i) {
            RV<NV> N;
            load(i + 2, N);  // row i + 2 in flight across row i's arithmetic
            load_prev(i + 1, qx, qy);
            sweep1(i, G1, G2, G3, px, py, S2);
            if (kK == 2 && i - 1 >= r0 && i - 1 < r1) {
                // sweep 2 of row i - 1 from the x_{k+1} rows S0 (i - 2), S1 (i - 1), S2 (i)
                const int iv = i - 1;
                GradAcc<NV> A = vertex_sums<NV>(S0, S1, S2, hl, hr, iv > 0, iv < g.nv - 1);
                if (own) {
                    const int64_t o = (int64_t)iv * g.nh + ih;
                    const int64_t r = ring_pos(g, iv, ih);
                    if (r >= 0) {  // k_gd_grad_ring adds the chords of x_{k+1} and solves
                        acc_store<NV>(a.ring_acc + r * kAccWords(NV), A);
                    } else {
#pragma unroll
                        for (int v = 0; v < NV; ++v) {
                            const VConst k = vertex_consts<NV>(A, v);
                            double y0, y1;
                            jacobi_y(k, A.s0[v], A.s1[v], y0, y1);
                            worst2 = fmax(worst2, change_of(S1.gx[v], S1.gy[v], y0, y1));
                            // Chebyshev against x_k of row i - 1 (G1)
                            a.gout2[2 * (v * n + o)] = cheb(st2, y0, G1.gx[v]);
                            a.gout2[2 * (v * n + o) + 1] = cheb(st2, y1, G1.gy[v]);
                        }
                    }
                }
            }
            G0 = G1;
            G1 = G2;
            G2 = G3;
            G3 = N;
            S0 = S1;
            S1 = S2;
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                px[v] = qx[v];
                py[v] = qy[v];
            }
        }
    }
    // the two sweeps' largest changes: wave reduction, one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        worst1 = fmax(worst1, __shfl_down(worst1, off));
        worst2 = fmax(worst2, __shfl_down(worst2, off));
    }
    if (lane == 0 && a.chg) {
        const unsigned long long b1 = (unsigned long long)__double_as_longlong(worst1);
        if (worst1 > 0 && __hip_atomic_load(&a.chg[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < b1)
            atomicMax(&a.chg[0], b1);
        const unsigned long long b2 = (unsigned long long)__double_as_longlong(worst2);
        if (kK == 2 && worst2 > 0 && __hip_atomic_load(&a.chg[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < b2)
            atomicMax(&a.chg[1], b2);
    }
}

// ------------------------------------------------------------------ cone solve (fixed K sweeps)
//
// After K Chebyshev sweeps from x_0 = 0 a vertex's gradient depends only on the vertices within K
// hops of it (each sweep reads the 1-hop neighbours' previous iterate and the vertex's own
// iterate before that). The interpolated values need the gradients at the vertices of the
// triangles that hold targets only, so for a 128^2 target grid over a 1e7-point lattice the global
// iteration's x_K there is formed from small patches instead of K passes over the whole lattice:
//   * interior targets (their cell more than K + 1 cells from the lattice boundary): the
//     (2K + 4)^2 box around the cell in LDS, K sweeps on the shrinking square that still influences
//     the cell (x_j on the vertices within K + 1 - j of it), k_gd_cone_patch;
//   * the rest (cells near the boundary, pocket triangles): the ring's pocket chords couple vertices
//     far along a side, so those run the global iteration on the boundary band (depth <= 2K + 3 - j
//     at sweep j, one launch per sweep, the chords in 8-lane groups), valid to depth K + 3 after K
//     sweeps.
// Both use the gradient arithmetic above, so every target vertex holds the global iteration's
// K-sweep value bit for bit (tests/test_gpu_parity.py::test_gradient_cone_equals_global_sweeps).

constexpr int kConeMaxK = 14;                    // patch box side 2K + 4 <= 32
constexpr int kConeBox = 2 * kConeMaxK + 4;  // the largest box side: it fits the patches' LDS pitch

// the boundary band: vertices with min(iv, ih, nv - 1 - iv, nh - 1 - ih) <= D, as four regions -
// the top rows [0, rt), the bottom rows [rb, nv), and between them the left columns [0, cl) and the
// right columns [cr, nh) - cut into kBandTR x kBandTC tiles (every band vertex in one tile)
constexpr int kBandTR = 16, kBandTC = 32;  // (33 KB of LDS a tile, 126 VGPRs: a workgroup fits beside the passes')
struct BandTiles {
    int D, rt, rb, cl, cr;
    int ncb, top_rb, bot_rb, mid_rb, lcb, rcb;  // column blocks (top / bottom), row blocks, side column blocks
    int n_top, n_bot, n_left, total;            // tile counts (the right side's are the rest)
};

inline BandTiles band_tiles(int nv, int nh, int D) {
    BandTiles b{};
    b.D = D;
    b.rt = std::min(D + 1, nv);
    b.rb = std::max(nv - (D + 1), b.rt);
    b.cl = std::min(D + 1, nh);
    b.cr = std::max(nh - (D + 1), b.cl);
    auto cdiv = [](int a, int q) { return (a + q - 1) / q; };
    b.ncb = cdiv(nh, kBandTC);
    b.top_rb = cdiv(b.rt, kBandTR);
    b.bot_rb = cdiv(nv - b.rb, kBandTR);
    b.mid_rb = cdiv(b.rb - b.rt, kBandTR);
    b.lcb = cdiv(b.cl, kBandTC);
    b.rcb = cdiv(nh - b.cr, kBandTC);
    b.n_top = b.top_rb * b.ncb;
    b.n_bot = b.bot_rb * b.ncb;
    b.n_left = b.mid_rb * b.lcb;
    b.total = b.n_top + b.n_bot + b.n_left + b.mid_rb * b.rcb;
    return b;
}

// tile t's origin and its region's end: rows [r0, r1) x columns [c0, c1) of the tile's vertices
__device__ __forceinline__ void band_tile(const BandTiles& b, int nv, int nh, int t, int& r0, int& c0, int& r1,
                                          int& c1) {
    if (t < b.n_top) {
        r0 = (t / b.ncb) * kBandTR;
        c0 = (t % b.ncb) * kBandTC;
        r1 = b.rt;
        c1 = nh;
    } else if ((t -= b.n_top) < b.n_bot) {
        r0 = b.rb + (t / b.ncb) * kBandTR;
        c0 = (t % b.ncb) * kBandTC;
        r1 = nv;
        c1 = nh;
    } else if ((t -= b.n_bot) < b.n_left) {
        r0 = b.rt + (t / b.lcb) * kBandTR;
        c0 = (t % b.lcb) * kBandTC;
        r1 = b.rb;
        c1 = b.cl;
    } else {
        t -= b.n_left;
        r0 = b.rt + (t / b.rcb) * kBandTR;
        c0 = b.cr + (t % b.rcb) * kBandTC;
        r1 = b.rb;
        c1 = nh;
    }
    r1 = min(r1, r0 + kBandTR);
    c1 = min(c1, c0 + kBandTC);
}

struct ConeBand {
    const double* f;      // (n) one value set
    const double* gin;    // x_{j-1} (n, 2) or nullptr (x_0 = 0)
    const double* gprev;  // x_{j-2} (mode 2)
    double* gout;         // x_j
    ConeStep st;
    const int* needed;    // device flag: some target needs the band (else the launch returns at once)
    unsigned long long* clk = nullptr;  // diagnostics (or nullptr): the ring-only / tile workgroups' wall-clock
                                        // time summed, their counts, their longest (akb_gd_patch_phases)
    const int32_t* slots = nullptr;     // (L, 8): ring vertex r's chord neighbours padded with -1 (or nullptr)
};

// the lattice edges of a band vertex in the fixed order (left, right, down, up, the diagonals), from
// its neighbours' data - the one arithmetic of the gather kernel and the tiles
__device__ __forceinline__ void band_edges(GradAcc<1>& A, double xi, double yi, double fi, const double (&xs)[8],
                                           const double (&ys)[8], const double (&fs)[8], const double (&gxs)[8],
                                           const double (&gys)[8], const bool (&on)[8]) {
    const double fi1[1] = {fi};
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if (on[k]) {
            const double fj[1] = {fs[k]}, gxj[1] = {gxs[k]}, gyj[1] = {gys[k]};
            if (k < 4) acc_edge<1, false>(A, edge_geom(xs[k] - xi, ys[k] - yi), fi1, fj, gxj, gyj);
            else acc_edge<1, true>(A, edge_geom(xs[k] - xi, ys[k] - yi), fi1, fj, gxj, gyj);
        }
    acc_fold<1>(A);
}

// vertex i's lattice-edge sums of one band sweep: every candidate neighbour's data loaded first
// (positions off the lattice clamped to i, the diagonals' presence from their cells' bytes, loaded
// beside them), then the edges in order: one memory round trip per vertex instead of one per edge
__device__ __forceinline__ void band_grid_sums(const Grid& g, const ConeBand& a, int64_t i, int iv, int ih,
                                               double xi, double yi, double fi, GradAcc<1>& A) {
    const int64_t nh = g.nh;
    const bool L = ih > 0, R = ih < g.nh - 1, D = iv > 0, U = iv < g.nv - 1;
    const int64_t jn[8] = {i - 1, i + 1, i - nh, i + nh, i - nh - 1, i - nh + 1, i + nh - 1, i + nh + 1};
    const bool inb[8] = {L, R, D, U, D && L, D && R, U && L, U && R};
    const int64_t c0 = (int64_t)iv * (g.nh - 1) + ih;
    const int64_t dc[4] = {c0 - g.nh, c0 - (g.nh - 1), c0 - 1, c0};
    uint8_t dg[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) dg[k] = g.diag[inb[4 + k] ? dc[k] : 0];
    double xs[8], ys[8], fs[8], gxs[8], gys[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int64_t j = inb[k] ? jn[k] : i;
        xs[k] = g.x[j];
        ys[k] = g.y[j];
        fs[k] = a.f[j];
        gxs[k] = a.gin ? a.gin[2 * j] : 0.0;
        gys[k] = a.gin ? a.gin[2 * j + 1] : 0.0;
    }
    const bool on[8] = {L, R, D, U, inb[4] && dg[0] == 0, inb[5] && dg[1] == 1, inb[6] && dg[2] == 1,
                        inb[7] && dg[3] == 0};
    band_edges(A, xi, yi, fi, xs, ys, fs, gxs, gys, on);
}

// the solve of one band / ring vertex of sweep j, stored to x_j (px, py: x_{j-2} there, mode 2)
__device__ __forceinline__ void band_solve(const ConeBand& a, int64_t i, const GradAcc<1>& A, double px, double py) {
    const VConst k = vertex_consts<1>(A, 0);
    double y0, y1;
    jacobi_y(k, A.s0[0], A.s1[0], y0, y1);
    const int64_t o = 2 * i;
    a.gout[o] = cheb(a.st, y0, px);
    a.gout[o + 1] = cheb(a.st, y1, py);
}
__device__ __forceinline__ void band_solve(const ConeBand& a, int64_t i, const GradAcc<1>& A) {
    const int64_t o = 2 * i;
    band_solve(a, i, A, a.st.mode == 2 ? a.gprev[o] : 0.0, a.st.mode == 2 ? a.gprev[o + 1] : 0.0);
}

// ring vertex r of a band sweep over a group of W lanes (sub: the lane in it): the pocket chords
// (chord_sums: each lane a strided part, the group's butterfly), then the lead lane adds the
// vertex's lattice-edge sums and solves
// the ring's chord slot table for the band sweeps, kChordSlots a vertex: a vertex of at most eight
// chords has them in xidx order (-1 past them); one of nine to kChordSlots has them encoded
// -(j + 3) (-1 past them), so a lane's first slot tells it the vertex is big; one of more has
// kSlotBig in every slot (the xptr path, a wave for the vertex)
constexpr int kChordSlots = 32;
constexpr int32_t kSlotBig = -2;
__device__ __forceinline__ int32_t slot_chord(int32_t v) { return v >= 0 ? v : v <= -3 ? -v - 3 : -1; }

template <int W>
__device__ __forceinline__ void cone_ring_vertex(const Grid& g, const ConeBand& a, int64_t r, int sub,
                                                 const int32_t (&js)[4] = {-1, -1, -1, -1}) {
    const int64_t n = (int64_t)g.nv * g.nh;
    const int64_t i = ring_vertex(g, r);
    // every load that needs only r first: the vertex, x_{j-2} there and the lattice neighbours (with
    // the slot table the chords came with the vertex's big test, so their data is in flight with
    // them: two memory latencies for the vertex)
    const double xi = g.x[i], yi = g.y[i];
    const double fi[1] = {a.f[i]};
    const bool pre = a.st.mode == 2 && sub == 0;
    const double ppx = pre ? a.gprev[2 * i] : 0.0, ppy = pre ? a.gprev[2 * i + 1] : 0.0;
    const bool slotted = W == 8 && a.slots;
    GradAcc<1> D;
    if (sub == 0) {
        const int iv = (int)(i / g.nh), ih = (int)(i - (int64_t)iv * g.nh);
        band_grid_sums(g, a, i, iv, ih, xi, yi, fi[0], D);
    }
    GradAcc<1> A;
    if (slotted) {
        auto chord = [&](int32_t c, GradAcc<1>& C) {
            if (c >= 0) {
                const double fj[1] = {a.f[c]}, gxj[1] = {a.gin ? a.gin[2 * (int64_t)c] : 0.0},
                             gyj[1] = {a.gin ? a.gin[2 * (int64_t)c + 1] : 0.0};
                acc_edge<1>(C, edge_geom(g.x[c] - xi, g.y[c] - yi), fi, fj, gxj, gyj);
            }
        };
        if (js[0] <= -3) {
            // nine to 32 chords: chord_sums<1, 64>'s lanes sub, sub + 8, ..., sub + 56 (a chord each,
            // zeros past them) combined as its butterfly's first three levels combine them, then the
            // group's butterfly its last three - the 64-lane path's bits, without a wave per vertex
            GradAcc<1> c0, c8, c16, c24;
            const GradAcc<1> z;
            chord(slot_chord(js[0]), c0);
            chord(slot_chord(js[1]), c8);
            chord(slot_chord(js[2]), c16);
            chord(slot_chord(js[3]), c24);
            acc_add<1>(c0, z);    // lane sub + 32
            acc_add<1>(c16, z);   // lane sub + 48
            acc_add<1>(c0, c16);  // (lane sub) + (lane sub + 16)
            acc_add<1>(c8, z);
            acc_add<1>(c24, z);
            acc_add<1>(c8, c24);
            acc_add<1>(c0, c8);
            A = c0;
        } else {  // at most eight: one chord a lane (chord_sums<1, 8>'s order)
            chord(js[0], A);
        }
        acc_reduce<1, W>(A);
    } else {
        A = chord_sums<1, W, W == 64 ? 1 : 4>(g, n, r, sub, xi, yi, fi, a.f, a.gin);
    }
    if (sub == 0) {
        acc_add<1>(A, D);
        band_solve(a, i, A, ppx, ppy);
    }
}

__global__ void k_gd_chord_slots(Grid g, int32_t* slots, int64_t L) {
    AKB_CHAIN_PRIORITY();
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < L; r += (int64_t)gridDim.x * blockDim.x) {
        const int32_t k0 = g.xptr[r], cnt = g.xptr[r + 1] - k0;
        int32_t* sr = slots + r * kChordSlots;
        for (int k = 0; k < kChordSlots; ++k)
            sr[k] = cnt > kChordSlots ? kSlotBig
                    : k >= cnt        ? -1
                    : cnt > 8         ? -g.xidx[k0 + k] - 3
                                      : g.xidx[k0 + k];
    }
}

// one sweep of the band in one launch, one round of 256-thread workgroups (a wave per SIMD, so a
// workgroup fits beside a pass-2 workgroup's four waves a SIMD instead of waiting for a CU to drain):
// the first ceil(L / 32) take ring vertices [32 b, 32 b + 32) (8-lane groups: a vertex's chords over
// the group, its lattice edges on the lead lane; a vertex of more than 32 chords takes its whole wave
// afterwards), the others band tile b - ceil(L / 32) - the tile's vertices and their neighbours' x,
// y, f and x_{j-1} (and the cells' diagonals), and x_{j-2} of its vertices, staged in LDS with
// coalesced row loads, then four vertices a thread off the ring (band_edges from LDS: the gather
// kernel's arithmetic). Both read x_{j-1} / x_{j-2} only.
constexpr int kBandThreads = 256, kBandRingWaves = kBandThreads / 64, kBandRingPer = 8 * kBandRingWaves;
constexpr int kBandTileThreads = kBandThreads, kBandVR = kBandTR * kBandTC / kBandTileThreads;
// a workgroup's wall-clock time into the diagnostics words (ring only: k = 0, with a tile: k = 1)
__device__ __forceinline__ void band_clock(unsigned long long* clk, int k, unsigned long long t0) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long d = wall_clock64() - t0;
        atomicAdd(&clk[2 * k], d);
        atomicAdd(&clk[2 * k + 1], 1ull);
        atomicMax(&clk[4 + k], d);
    }
}
// the band launch's ring workgroups (the tiles' follow them)
inline unsigned band_ring_wgs(int64_t L) { return (unsigned)((L + kBandRingPer - 1) / kBandRingPer); }
inline unsigned band_grid(const BandTiles& bt, int64_t L) { return band_ring_wgs(L) + (unsigned)bt.total; }

__global__ void __launch_bounds__(kBandThreads) __attribute__((amdgpu_waves_per_eu(4))) k_gd_cone_band(Grid g, BandTiles bt, ConeBand a) {
    AKB_CHAIN_PRIORITY();
    if (!*a.needed) return;
    const unsigned long long t0 = a.clk ? wall_clock64() : 0;
    constexpr int HR = kBandTR + 2, HC = kBandTC + 2, HN = HR * HC, CC = kBandTC + 1;
    __shared__ double sx[HN], sy[HN], sf[HN], sgx[HN], sgy[HN];
    __shared__ double spx[kBandTR * kBandTC], spy[kBandTR * kBandTC];  // x_{j-2} of the tile's vertices
    __shared__ uint8_t sdg[(kBandTR + 1) * CC];
    const int64_t L = 2 * (int64_t)(g.nh - 1) + 2 * (int64_t)(g.nv - 1);
    const int nr = (int)((L + kBandRingPer - 1) / kBandRingPer);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if ((int)blockIdx.x < nr) {  // (workgroup-uniform) ring vertices
        const int sub = lane & 7;
        const int64_t q0 = (int64_t)blockIdx.x * kBandRingPer + 8 * w;
        const int64_t r = q0 + (lane >> 3);
        int32_t js[4] = {-1, -1, -1, -1};
        bool big;
        if (a.slots) {  // the slots say whether the vertex is big: no xptr level ahead of the vertex's loads
            if (r < L) {
#pragma unroll
                for (int k = 0; k < 4; ++k) js[k] = a.slots[r * kChordSlots + sub + 8 * k];
            }
            big = js[0] == kSlotBig;
        } else {
            big = r < L && g.xptr[r + 1] - g.xptr[r] > 8;
        }
        if (r < L && !big) cone_ring_vertex<8>(g, a, r, sub, js);
        unsigned long long m = __ballot(big && sub == 0);
        while (m) {  // wave-uniform
            const int q = __builtin_ctzll(m);
            m &= m - 1;
            cone_ring_vertex<64>(g, a, q0 + (q >> 3), lane);
        }
        if (a.clk) band_clock(a.clk + 4, 0, t0);
        return;
    }
    int r0 = 0, c0 = 0, r1 = 0, c1 = 0;
    band_tile(bt, g.nv, g.nh, (int)blockIdx.x - nr, r0, c0, r1, c1);
    {
        // the tile's vertices with a one-vertex halo (rows r0 - 1 .. r0 + TR, inside the lattice), the
        // diagonals of cells (r0 - 1 .. r0 + TR - 1) x (c0 - 1 .. c0 + TC - 1) and x_{j-2} of the tile's
        // vertices: every load of a thread issued before the first LDS store (one memory latency)
        constexpr int NQ = (HN + kBandThreads - 1) / kBandThreads, NC = ((kBandTR + 1) * CC + kBandThreads - 1) / kBandThreads;
        constexpr int NP = kBandTR * kBandTC / kBandThreads;
        double lx[NQ], ly[NQ], lf[NQ], lgx[NQ], lgy[NQ], lpx[NP], lpy[NP];
        uint8_t ld[NC];
#pragma unroll
        for (int u = 0; u < NQ; ++u) {
            const int k = threadIdx.x + u * kBandThreads;
            const int iv = r0 - 1 + k / HC, ih = c0 - 1 + (k - (k / HC) * HC);
            lx[u] = ly[u] = lf[u] = lgx[u] = lgy[u] = 0.0;
            if (k < HN && iv >= 0 && iv < g.nv && ih >= 0 && ih < g.nh) {
                const int64_t q = (int64_t)iv * g.nh + ih;
                lx[u] = g.x[q];
                ly[u] = g.y[q];
                lf[u] = a.f[q];
                lgx[u] = a.gin ? a.gin[2 * q] : 0.0;
                lgy[u] = a.gin ? a.gin[2 * q + 1] : 0.0;
            }
        }
#pragma unroll
        for (int u = 0; u < NC; ++u) {
            const int k = threadIdx.x + u * kBandThreads;
            const int cv = r0 - 1 + k / CC, ch = c0 - 1 + (k - (k / CC) * CC);
            ld[u] = (k < (kBandTR + 1) * CC && cv >= 0 && cv < g.nv - 1 && ch >= 0 && ch < g.nh - 1)
                        ? g.diag[(int64_t)cv * (g.nh - 1) + ch] : 0;
        }
#pragma unroll
        for (int u = 0; u < NP; ++u) {
            const int k = threadIdx.x + u * kBandThreads;
            const int iv = r0 + k / kBandTC, ih = c0 + (k - (k / kBandTC) * kBandTC);
            lpx[u] = lpy[u] = 0.0;
            if (a.st.mode == 2 && iv < r1 && ih < c1) {
                const int64_t o = 2 * ((int64_t)iv * g.nh + ih);
                lpx[u] = a.gprev[o];
                lpy[u] = a.gprev[o + 1];
            }
        }
#pragma unroll
        for (int u = 0; u < NQ; ++u) {
            const int k = threadIdx.x + u * kBandThreads;
            if (k < HN) {
                sx[k] = lx[u];
                sy[k] = ly[u];
                sf[k] = lf[u];
                sgx[k] = lgx[u];
                sgy[k] = lgy[u];
            }
        }
#pragma unroll
        for (int u = 0; u < NC; ++u) {
            const int k = threadIdx.x + u * kBandThreads;
            if (k < (kBandTR + 1) * CC) sdg[k] = ld[u];
        }
#pragma unroll
        for (int u = 0; u < NP; ++u) {
            const int k = threadIdx.x + u * kBandThreads;
            spx[k] = lpx[u];
            spy[k] = lpy[u];
        }
        __syncthreads();
    }
    const int tt = threadIdx.x;
    const int tr0 = tt / kBandTC, tc = tt - (tt / kBandTC) * kBandTC;
#pragma unroll 1
    for (int u = 0; u < kBandVR; ++u) {
        const int tr = tr0 + u * (kBandTR / kBandVR);
        const int iv = r0 + tr, ih = c0 + tc;
        if (iv >= r1 || ih >= c1 || ring_pos(g, iv, ih) >= 0) continue;
        const bool L_ = ih > 0, R = ih < g.nh - 1, D = iv > 0, U = iv < g.nv - 1;
        const int li = (tr + 1) * HC + (tc + 1);
        const int jn[8] = {li - 1, li + 1, li - HC, li + HC, li - HC - 1, li - HC + 1, li + HC - 1, li + HC + 1};
        const bool inb[8] = {L_, R, D, U, D && L_, D && R, U && L_, U && R};
        const int lc = tr * CC + tc;  // cell (iv - 1, ih - 1)
        const int dc[4] = {lc, lc + 1, lc + CC, lc + CC + 1};
        uint8_t dg[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) dg[k] = inb[4 + k] ? sdg[dc[k]] : 0;
        double xs[8], ys[8], fs[8], gxs[8], gys[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int j = inb[k] ? jn[k] : li;
            xs[k] = sx[j];
            ys[k] = sy[j];
            fs[k] = sf[j];
            gxs[k] = sgx[j];
            gys[k] = sgy[j];
        }
        const bool on[8] = {L_, R, D, U, inb[4] && dg[0] == 0, inb[5] && dg[1] == 1, inb[6] && dg[2] == 1,
                            inb[7] && dg[3] == 0};
        GradAcc<1> A;
        band_edges(A, sx[li], sy[li], sf[li], xs, ys, fs, gxs, gys, on);
        const int pk = tr * kBandTC + tc;
        band_solve(a, (int64_t)iv * g.nh + ih, A, spx[pk], spy[pk]);
    }
    if (a.clk) band_clock(a.clk + 4, 1, t0);
}

struct ConePatch {
    const double* f;           // (n) one value set
    const int64_t* cells;      // interior target cells (duplicates allowed)
    const int* count;          // how many (device)
    int K;
    ConeStep st[kConeMaxK + 1];  // st[j] for sweep j = 1 .. K
    double* gout;              // x_K (n, 2): the cells' four corners are written
    unsigned long long* chg;   // largest change measure of one more sweep at the corners (or nullptr)
    unsigned long long* est;   // largest value-error estimate of a cell (or nullptr; see below)
    unsigned long long* clk;   // diagnostics (or nullptr): workgroup 0's wall clock in its steps' phases -
                               // setup, sweeps, the rest - summed, and its step count
};

// The patch threads' vertices (r | c << 8 per thread, 0xffff for the corner-store and idle threads),
// per K: each thread set holds its vertices in order of depth from the centre outwards, so that a
// sweep's shrinking square stays (nearly) a prefix of the set's threads, but reordered so that the
// sweeps' 16-byte LDS reads do not collide on banks. A ds_read_b128 serves a wave in four groups of
// 16 lanes (MI355X_MICROARCH.md §LDS), and with the box pitch P = 33 == 1 (mod 16) a vertex's read
// lands on the bank quad (r + c + slot offset) mod 16: a group is conflict-free when its vertices'
// r + c differ mod 16. Rings in depth order walk r + c up and then back down, and the small inner
// rings hold few residues, which cost 1.8x the conflict-free read cycles; the host picks each
// thread's vertex greedily from the next 32 of the depth order - the earliest whose residue is
// free in the thread's lane group (and, for the setup's 8-byte reads, mod 32 in its half-wave) -
// 1.1x (a vertex may so sit a few threads past shallower ones: the sweeps test depth per thread).
__constant__ uint16_t c_patch_order[kConeMaxK + 1][1024];

inline int b128_lane_group(int lane) {  // ds_read_b128's groups: {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, ...
    const int x = lane & 31;
    const bool first = x < 4 || (x >= 12 && x < 16) || (x >= 20 && x < 28);
    return (lane >> 5) * 2 + (first ? 0 : 1);
}

inline void patch_order_table(int K, int S, uint16_t* out) {
    const int W = 2 * K + 4, N2 = (W - 2 * S - 2) * (W - 2 * S - 2);
    for (int t = 0; t < 1024; ++t) out[t] = 0xffff;
    uint32_t used16[16][4] = {}, used32[16][2] = {};  // per wave: residues taken in each lane group / half
    struct V {
        int r, c, d;
    };
    for (int set = 0; set < 3; ++set) {  // inner A, inner B (depth >= S + 1), outer (depth 1 .. S)
        const int dhi = set < 2 ? K + 1 : S, dlo = set < 2 ? S + 1 : 1;
        V seq[1024];
        int n = 0;
        for (int d = dhi; d >= dlo; --d) {  // ring d clockwise from its top-left vertex
            const int s1 = W - 2 * d - 1;
            for (int i = 0; i < 4 * s1; ++i) {
                const int q = i / s1, e = i - q * s1;
                const int r = q == 0 ? d : q == 1 ? d + e : q == 2 ? d + s1 : d + s1 - e;
                const int c = q == 0 ? d + e : q == 1 ? d + s1 : q == 2 ? d + s1 - e : d;
                seq[n++] = V{r, c, d};
            }
        }
        int pos = set == 0 ? 0 : set == 1 ? N2 : 2 * N2, head = 0;
        while (head < n) {
            const int w = pos >> 6, l = pos & 63, grp = b128_lane_group(l), h = l >> 5;
            int best = head;
            if (seq[head].d != K + 1) {  // (the innermost ring, the corners, stays the set's first four)
                int bs = 1 << 30;
                for (int k = head; k < std::min(n, head + 32); ++k) {
                    const int rc = seq[k].r + seq[k].c;
                    const int sc = (int)((used16[w][grp] >> (rc & 15)) & 1) * 100000 +
                                   (int)((used32[w][h] >> (rc & 31)) & 1) * 10000 + (k - head);
                    if (sc < bs) {
                        bs = sc;
                        best = k;
                    }
                }
            }
            const V v = seq[best];
            for (int k = best; k > head; --k) seq[k] = seq[k - 1];  // the rest keep their order
            ++head;
            used16[w][grp] |= 1u << ((v.r + v.c) & 15);
            used32[w][h] |= 1u << ((v.r + v.c) & 31);
            out[pos++] = (uint16_t)(v.r | (v.c << 8));
        }
    }
}

// the patches' split S for K (the smallest S >= K / 2 with the three thread sets - two inner, one
// outer - and the four corner-store threads in one workgroup), or -1
inline int patch_split(int K) {
    const int W = 2 * K + 4;
    for (int s2 = (K + 1) / 2; s2 <= K; ++s2)
        if ((W - 2) * (W - 2) + (W - 2 * s2 - 2) * (W - 2 * s2 - 2) + 4 <= 1024) return s2;
    return -1;
}

// every K's table into the constant memory of the device stream s runs on, once per device and
// process (before that device's first patch launch: a module's constant memory is per device, and
// the thread-per-GPU callers run the solve on several devices from one process)
inline int patch_order_upload(hipStream_t s) {
    static std::mutex mu;
    static uint16_t tab[kConeMaxK + 1][1024];
    static bool built = false;
    static uint64_t done = 0;  // devices (bit d) whose copy holds the tables
    int dev = 0, cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return 1;
    dev = cur;
    if (s != nullptr && hipStreamGetDevice(s, &dev) != hipSuccess) return 1;
    if (dev < 0 || dev >= 64) return 1;
    std::lock_guard<std::mutex> lk(mu);
    if ((done >> dev) & 1u) return 0;
    if (!built) {
        for (int K = 0; K <= kConeMaxK; ++K) {
            const int S = K >= 1 ? patch_split(K) : -1;
            if (S >= 0) patch_order_table(K, S, tab[K]);
            else std::fill(tab[K], tab[K] + 1024, (uint16_t)0xffff);
        }
        built = true;
    }
    if (dev != cur && hipSetDevice(dev) != hipSuccess) return 1;
    const bool ok = hipMemcpyToSymbol(HIP_SYMBOL(c_patch_order), tab, sizeof(tab)) == hipSuccess;
    if (dev != cur) (void)hipSetDevice(cur);
    if (!ok) return 1;
    done |= 1ull << dev;
    return 0;
}

// The interior target cells' patches: one persistent workgroup per CU walks its cells as a
// two-stage pipeline. A thread holds one box vertex (the box has pitch 33 in LDS) and that
// vertex's constants - the eight edge slots' M (zero for an absent diagonal) and c, P - in
// registers, so a sweep costs eight LDS reads and 4 FMAs per slot plus the 2 x 2 product and the
// Chebyshev step. Three thread sets, in order of depth from the centre outwards within each:
//   * inner A = threads [0, N2), inner B = [N2, 2 N2): the N2 = (W - 2S - 2)^2 vertices of depth
//     >= S + 1, the ones the late sweeps S + 1 .. K still update;
//   * outer = [2 N2, N1 + N2): the vertices of depth 1 .. S (N1 = (W - 2)^2 of depth >= 1 in all).
// (Within a set the vertices are permuted against LDS bank conflicts, c_patch_order.)
// Step p sets cell p up on the outer threads and on inner set p & 1, which run its sweeps 1 .. S;
// the other inner set, whose registers still hold cell p - 1's constants from the step before,
// runs that cell's sweeps S + 1 .. K and its corners' output beside them. So every vertex's
// constants are formed once per cell, and the late sweeps (a few waves each) never run alone.
// A sweep's shrinking square is a prefix of each set's threads. Sweep 1 reads nothing: x_0 = 0
// makes S = +0, the same bits as summing the zero iterate, so each fresh thread runs it right
// after its constants, and the old set runs its sweep S + 1 (its own iterate only) during that
// setup: the barrier-separated loop then holds max(S - 1, K - S - 1) sweeps. A box whose cells all take the same
// diagonal (about two in three at C3) runs the sweeps over its six present slots (an absent
// slot adds exact zeros, so the bits are the eight-slot sum's); a wave reads that from the
// boxes' orientation words. Box sets of x, y, f rotate over two (cell p's, read by its setup;
// cell p + 1's, loaded through registers during the sweeps and written after them: the old set
// keeps the little geometry its corners need in registers), iterate pairs over two (cell p - 1's
// x_S, x_{S-1} stay where its sweeps left them). The host picks S (the smallest >= K/2 with
// N1 + N2 + 4 threads in a workgroup: threads N1 + N2 .. + 3 store the corners).
//
// At the corners (x_K) the kernel also forms the change one more plain sweep would make - scipy's
// measure (chg) - and a value-error estimate: with the Jacobi spectrum in [-1/2, 1/2] the distance
// of x_K from the fixed point is at most ~2x the step |y - x_K|, and a Clough-Tocher value moves
// by at most |dg| x the longest edge it integrates over, so est = 2 sqrt2 max|y - x_K| x the cell's
// longest side or diagonal (in the map's units; FaithfulPupil checks it against the map's range).
// A NaN step makes the estimate NaN, which the max keeps (fmax would drop it) and the guard
// refuses.
__device__ __forceinline__ double nan_max(double a, double b) { return (a != a || b != b) ? (a + b) : fmax(a, b); }

__device__ __forceinline__ double cell_est(const double (&so)[4][6]) {
    const double d = nan_max(nan_max(so[0][4], so[1][4]), nan_max(so[2][4], so[3][4]));
    const double h = fmax(fmax(so[0][5], so[1][5]), fmax(so[2][5], so[3][5]));
    return 2.0 * 1.4142135623730951 * d * h;
}

// the patch workgroup's size for K and S (every vertex thread, the four corner-store threads, and
// the 32-wide box-load rows)
__host__ __device__ constexpr int patch_threads(int K, int S) {
    return ((((2 * K + 2) * (2 * K + 2) + (2 * K + 2 - 2 * S) * (2 * K + 2 - 2 * S) + 4) >
                     32 * (2 * K + 4)
                 ? ((2 * K + 2) * (2 * K + 2) + (2 * K + 2 - 2 * S) * (2 * K + 2 - 2 * S) + 4)
                 : 32 * (2 * K + 4)) +
            63) &
           ~63;
}

// S of one sweep: the slots of kMask (bit k: slot k) summed from the iterate at gi (the vertex's
// buffer entry, minus P + 1 so that every slot's offset is a positive immediate), in the fixed
// order - the axis chain s, the diagonal chain d - then s + d
template <int kMask, int P>
__device__ __forceinline__ void patch_sums(const double2* __restrict__ buf, int i0, const double (&mxx)[8],
                                           const double (&mxy)[8], const double (&myy)[8], double& s0, double& s1) {
    constexpr int off[8] = {P, P + 2, 1, 2 * P + 1, 0, 2, 2 * P, 2 * P + 2};
    asm volatile("" : "+v"(i0));  // i0 = b - P - 1 as computed: the slots' offsets stay immediates
    double2 gj[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if (kMask & (1 << k)) gj[k] = buf[i0 + off[k]];
    double a0 = 0.0, a1 = 0.0, d0 = 0.0, d1 = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (!(kMask & (1 << k))) continue;
        double& t0 = k < 4 ? a0 : d0;
        double& t1 = k < 4 ? a1 : d1;
        t0 = __builtin_fma(mxy[k], gj[k].y, __builtin_fma(mxx[k], gj[k].x, t0));
        t1 = __builtin_fma(myy[k], gj[k].y, __builtin_fma(mxy[k], gj[k].x, t1));
    }
    s0 = a0 + d0;
    s1 = a1 + d1;
}
constexpr int kSlotsAll = 0xff, kSlotsDiag0 = 0x9f, kSlotsDiag1 = 0x6f;  // diagonal 0: slots 4, 7; 1: 5, 6

__global__ void __launch_bounds__(1024) k_gd_cone_patch(Grid g, ConePatch a, int S) {
    constexpr int P = 33;
    static_assert(kConeBox < P, "box pitch");
    __shared__ double sxyf[2][3][P * 32];
    __shared__ double2 sg[2][2][P * 32];
    __shared__ uint8_t sd[2][P * 32];
    __shared__ int2 scell[1024];   // this workgroup's cells' box origins (R0, C0), read once
    __shared__ double sout[4][6];  // the old set's corner results, stored one step later
    __shared__ unsigned sori[2];   // per box set: bit 0 some cell takes diagonal 0, bit 1 some diagonal 1
    __shared__ double somg[kConeMaxK + 1];  // sweep j's Chebyshev weight
    __shared__ double shc[2][4];   // per iterate pair: the corners' longest cell side or diagonal
    __shared__ double smax[2];     // the corners' running maxima over this workgroup's cells: change, estimate
    const int K = a.K, W = 2 * K + 4;
    const int t = threadIdx.x;
    const int N1 = (W - 2) * (W - 2), N2 = (W - 2 * S - 2) * (W - 2 * S - 2), T0 = N1 + N2;
    const int role = t < N2 ? 0 : t < 2 * N2 ? 1 : t < T0 ? 2 : 3;  // inner A, inner B, outer, corner / idle
    int r = -1, c = -1, dep = 0;
    if (role < 3) {
        const unsigned v = c_patch_order[K][t];
        r = (int)(v & 0xffu);
        c = (int)(v >> 8);
        dep = min(min(r, c), min(W - 1 - r, W - 1 - c));
    }
    const int b = dep >= 1 ? r * P + c : P + 1;  // (idle threads: a harmless in-range base)
    const int Q = max(S - 1, K - S - 1);  // the step loop's sweeps (sweeps 1 and S + 1 run beside the setup)
    const int count = *a.count;
    const int my = count > (int)blockIdx.x ? (count - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    const double* const gx_ = g.x;
    const double* const gy_ = g.y;
    const double* const gf_ = a.f;
    const uint8_t* const gd_ = g.diag;
    const int nh = g.nh;
    // the cell list into LDS first (the host keeps it <= 1024 cells per workgroup), so no wait on a
    // global load sits between a step's barrier and its setup
    for (int i = t; i < my; i += blockDim.x) {
        const int64_t cell = a.cells[blockIdx.x + (int64_t)i * gridDim.x];
        const int iv0 = (int)(cell / (nh - 1)), ih0 = (int)(cell - (int64_t)iv0 * (nh - 1));
        scell[i] = make_int2(iv0 - (K + 1), ih0 - (K + 1));
    }
    if (t < 2) {
        sori[t] = 0u;
        smax[t] = 0.0;
    }
    if (t <= kConeMaxK) somg[t] = a.st[t].omega;
    __syncthreads();
    // the box loaders' row and column: re-formed where used (from an opaque copy of t), so that their
    // addresses are not held in registers across the sweeps
    auto lrc = [&](int& lr, int& lc) {
        int tt = t;
        asm volatile("" : "+v"(tt));
        lr = tt >> 5;
        lc = tt & 31;
    };
    int lr, lc;
    lrc(lr, lc);
    const bool loader = lr < W && lc < W, cell_loader = lr < W - 1 && lc < W - 1;
    // cell 0's box through registers (every later box loads during the step before it)
    uint8_t pd = 0;
    if (my > 0 && loader) {
        const int2 o = scell[0];
        const int64_t q = (int64_t)(o.x + lr) * nh + (o.y + lc);
        sxyf[0][0][lr * P + lc] = gx_[q];
        sxyf[0][1][lr * P + lc] = gy_[q];
        sxyf[0][2][lr * P + lc] = gf_[q];
        if (cell_loader) pd = gd_[(int64_t)(o.x + lr) * (nh - 1) + (o.y + lc)];
    }
    constexpr int off[8] = {-1, 1, -P, P, -P - 1, -P + 1, P - 1, P + 1};
    const bool clk = a.clk && blockIdx.x == 0 && __builtin_amdgcn_readfirstlane(t >> 6) == 0;  // wave 0 (scalar)
    unsigned long long c_setup = 0, c_sweeps = 0, c_rest = 0, c0 = clk ? wall_clock64() : 0, c1 = 0;
    // the vertex's constants (kept across two steps by the inner sets), its box's orientation word and,
    // at a corner, the cell's longest side or diagonal there
    double mxx[8], mxy[8], myy[8];
    VConst kc{0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 8; ++k) mxx[k] = mxy[k] = myy[k] = 0.0;
    unsigned ori = 3u;
    for (int p = 0; p <= my; ++p) {
        const int s1 = p & 1;  // cell p's box set and iterate pair
        if (clk && p > 0) {  // the previous step's corners and next box writes
            const unsigned long long now = wall_clock64();
            c_rest += now - c0;
            c0 = now;
        }
        if (p < my && loader) {
            lrc(lr, lc);
            sd[s1][lr * P + lc] = pd;
        }
        {  // the box's diagonal orientations: one LDS atomic a wave
            const bool cv = p < my && cell_loader;
            const unsigned long long b0 = __ballot(cv && pd == 0), b1 = __ballot(cv && pd != 0);
            if ((t & 63) == 0 && (b0 | b1)) atomicOr(&sori[s1], (b0 ? 1u : 0u) | (b1 ? 2u : 0u));
        }
        // cell p's box came through registers to LDS last step: an LDS-only barrier, so no wave waits
        // here for the acks of its earlier global stores (__syncthreads' fence would)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (p >= 2 && role == 3 && t < T0 + 4) {  // cell p - 2's corners, left by the last step's old set
            const int q = t - T0;
            const int64_t i = (int64_t)sout[q][2];
            a.gout[2 * i] = sout[q][0];
            a.gout[2 * i + 1] = sout[q][1];
            if (q == 0) {  // the running maxima (in LDS: no register held across the steps)
                smax[0] = fmax(fmax(smax[0], fmax(sout[0][3], sout[1][3])), fmax(sout[2][3], sout[3][3]));
                smax[1] = nan_max(smax[1], cell_est(sout));
            }
        }
        const bool fresh = role == 2 || role == s1;  // this step: cell p (sweeps 1 .. S), else cell p - 1
        const bool act = dep >= 1 && (fresh ? p < my : p >= 1);
        double2(*const gg)[P * 32] = sg[fresh ? s1 : s1 ^ 1];  // this thread's cell's iterate pair
        // sweep j at this thread's vertex, its form the host's steps: 1 plain (x_0 = 0: S = +0, no
        // reads), 2 against x_0 = 0, later against x_{j-2}; w0 / w1: the wave's slot set is six slots
        // (every active lane's box takes one diagonal throughout)
        auto sweep = [&](int j, bool w0, bool w1) {
            const double om = somg[j];
            const int in = (j - 1) & 1, out = j & 1;
            const double2 pv = j >= 3 ? gg[out][b] : make_double2(0.0, 0.0);  // x_{j-2}, overwritten
            double s0 = 0.0, s1v = 0.0;
            if (j >= 2) {
                if (w0) patch_sums<kSlotsDiag0, P>(gg[in], b - P - 1, mxx, mxy, myy, s0, s1v);
                else if (w1) patch_sums<kSlotsDiag1, P>(gg[in], b - P - 1, mxx, mxy, myy, s0, s1v);
                else patch_sums<kSlotsAll, P>(gg[in], b - P - 1, mxx, mxy, myy, s0, s1v);
            }
            double y0, y1;
            jacobi_y(kc, s0, s1v, y0, y1);
            if (j == 1)
                gg[out][b] = make_double2(y0, y1);
            else
                gg[out][b] = make_double2(__builtin_fma(om, y0 - pv.x, pv.x), __builtin_fma(om, y1 - pv.y, pv.y));
        };
        if (act && fresh) {  // cell p's constants: the eight slots' M in the edge order, c and P
            const double* const sx = sxyf[s1][0];
            const double* const sy = sxyf[s1][1];
            const double* const sf = sxyf[s1][2];
            const uint8_t* const sdd = sd[s1];
            ori = sori[s1];
            const unsigned em = 0x0fu | (sdd[b - P - 1] == 0 ? 0x10u : 0u) | (sdd[b - P] == 1 ? 0x20u : 0u) |
                                (sdd[b - 1] == 1 ? 0x40u : 0u) | (sdd[b] == 0 ? 0x80u : 0u);
            const double xi = sx[b], yi = sy[b];
            const double fi[1] = {sf[b]}, zero[1] = {0.0};
            GradAcc<1> A;
            // every slot's neighbour read up front (the box holds them all): one LDS latency for the
            // eight, not one per present diagonal behind its branch
            double nx[8], ny[8], nf[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                nx[k] = sx[b + off[k]];
                ny[k] = sy[b + off[k]];
                nf[k] = sf[b + off[k]];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                mxx[k] = mxy[k] = myy[k] = 0.0;
                if (!(em & (1u << k))) continue;
                const EdgeG e = edge_geom(nx[k] - xi, ny[k] - yi);
                const double fj[1] = {nf[k]};
                acc_edge<1>(A, e, fi, fj, zero, zero);  // (its S part is not used: the sweeps form S)
                mxx[k] = e.mxx;
                mxy[k] = e.mxy;
                myy[k] = e.myy;
            }
            kc = vertex_consts<1>(A, 0);
            if (dep == K + 1) {  // a corner (the corners are (K+1 .. K+2)^2 of the box): the cell's two
                                 // sides and its diagonal there, for the value-error estimate
                int tb = t;
                asm volatile("" : "+v"(tb));  // (its addresses formed here, not held across the step)
                const int bq = b + (tb - t);
                const int dr = r == K + 1 ? P : -P, dc = c == K + 1 ? 1 : -1;
                auto l2 = [&](int j) {
                    const double ex = sx[j] - xi, ey = sy[j] - yi;
                    return ex * ex + ey * ey;
                };
                shc[s1][role == 0 ? t : t - N2] = sqrt(fmax(fmax(l2(bq + dr), l2(bq + dc)), l2(bq + dr + dc)));
            }
            sweep(1, false, false);  // reads nothing: no barrier between the constants and x_1
        } else if (act && S < K) {
            // the old set's first late sweep, S + 1, beside the setup (it reads only its own cell's
            // iterate pair, complete since the last step's sweeps): the step loop then runs
            // max(S - 1, K - S - 1) sweeps, one fewer than the two sets' sweep counts would need
            sweep(S + 1, __ballot(ori != 1u) == 0, __ballot(ori != 2u) == 0);
        }
        // cell p + 1's box point through registers: issued after the setup (whose temporaries then
        // are dead), written to LDS after the sweeps, which hide its latency
        double rx_ = 0.0, ry_ = 0.0, rf_ = 0.0;
        if (p + 1 < my) {
            pd = 0;
            const int2 o = scell[p + 1];
            if (loader) {
                lrc(lr, lc);
                const int64_t q = (int64_t)(o.x + lr) * nh + (o.y + lc);
                rx_ = gx_[q];
                ry_ = gy_[q];
                rf_ = gf_[q];
                if (cell_loader) pd = gd_[(int64_t)(o.x + lr) * (nh - 1) + (o.y + lc)];
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (t == 0) sori[s1 ^ 1] = 0u;  // cell p + 1's word (cell p - 1's was read in its own setup)
        if (clk) {
            c1 = wall_clock64();
            c_setup += c1 - c0;
        }
        // the wave's slot set: six slots when every active lane's box takes one diagonal throughout
        const bool w0 = __ballot(act && ori != 1u) == 0, w1 = __ballot(act && ori != 2u) == 0;
        for (int q = 1; q <= Q; ++q) {
            const int j = fresh ? q + 1 : S + 1 + q;
            if (act && dep >= j && j <= (fresh ? S : K)) sweep(j, w0, w1);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
        if (clk) {
            c0 = wall_clock64();
            c_sweeps += c0 - c1;
        }
        // cell p - 1's corners (the old set's innermost ring): x_K, the change of one more plain
        // sweep and the value-error estimate, into LDS; the corner-store threads store them after the
        // next step's barrier (or below, after the last step), so the stores' latency is not waited
        // for at the next step's top
        if (!fresh && act && dep == K + 1) {
            const int2 o = scell[p - 1];
            const int fin = K & 1;
            const double2 gk = gg[fin][b];
            double s0, s1v, y0, y1;
            patch_sums<kSlotsAll, P>(gg[fin], b - P - 1, mxx, mxy, myy, s0, s1v);
            jacobi_y(kc, s0, s1v, y0, y1);
            const int q = role == 0 ? t : t - N2;  // the innermost ring: a set's first four threads
            sout[q][0] = gk.x;
            sout[q][1] = gk.y;
            sout[q][2] = (double)((int64_t)(o.x + r) * nh + (o.y + c));
            sout[q][3] = a.chg ? change_of(gk.x, gk.y, y0, y1) : 0.0;
            sout[q][4] = nan_max(fabs(gk.x - y0), fabs(gk.y - y1));
            sout[q][5] = shc[s1 ^ 1][q];
        }
        if (p + 1 < my && loader) {  // set (p + 1) & 1 is read from the next step on
            lrc(lr, lc);
            const int q = lr * P + lc, st = s1 ^ 1;
            sxyf[st][0][q] = rx_;
            sxyf[st][1][q] = ry_;
            sxyf[st][2][q] = rf_;
        }
        if (p == my && my >= 1) {  // the last cell's corners
            __syncthreads();
            if (role == 3 && t < T0 + 4) {
                const int q = t - T0;
                const int64_t i = (int64_t)sout[q][2];
                a.gout[2 * i] = sout[q][0];
                a.gout[2 * i + 1] = sout[q][1];
                if (q == 0) {
                    smax[0] = fmax(fmax(smax[0], fmax(sout[0][3], sout[1][3])), fmax(sout[2][3], sout[3][3]));
                    smax[1] = nan_max(smax[1], cell_est(sout));
                }
            }
        }
    }
    if (t == T0) {
        const double cmax = smax[0], emax = smax[1];
        if (a.chg && cmax > 0) atomicMax(a.chg, (unsigned long long)__double_as_longlong(cmax));
        // a NaN estimate as +inf (ordered bits: the guard sees an estimate above any bar)
        if (a.est && (emax > 0 || emax != emax))
            atomicMax(a.est, (unsigned long long)__double_as_longlong(emax != emax ? HUGE_VAL : emax));
    }
    if (clk && t == 0) {
        a.clk[0] += c_setup;
        a.clk[1] += c_sweeps;
        a.clk[2] += c_rest;
        a.clk[3] += (unsigned long long)(my + 1);
    }
}

// targets -> interior target cells (the patch list) and whether any target needs the band
__global__ void __launch_bounds__(kBlock) k_gd_cone_targets(Grid g, const int* __restrict__ owner, int64_t m, int K,
                                                             int64_t* cells, int* count, int* band) {
    AKB_CHAIN_PRIORITY();
    const int64_t nc2 = 2 * ncells(g);
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < m; t += (int64_t)gridDim.x * blockDim.x) {
        const int o = owner[t];
        if (o == INT32_MAX) continue;
        bool interior = false;
        int64_t c = -1;
        if (o < nc2) {
            c = o >> 1;
            const int iv = (int)(c / (g.nh - 1)), ih = (int)(c - (int64_t)iv * (g.nh - 1));
            // the box rows iv - K - 1 .. iv + K + 2 clear of the ring rows / columns
            interior = iv - K - 1 >= 1 && iv + K + 2 <= g.nv - 2 && ih - K - 1 >= 1 && ih + K + 2 <= g.nh - 2;
        }
        if (interior) cells[atomicAdd(count, 1)] = c;
        else atomicOr(band, 1);
    }
}

// the driver's target grid axes from the lattice's extent (its extremes lie on the boundary ring):
// np.linspace(min, max, m) of the ring's x and y - i * step + start, the last point the stop
// (numpy 2.x's linspace arithmetic) - one workgroup
constexpr int kAxesThreads = 1024;  // one workgroup over the ring (4 x kBlock: the loop was its latency)
constexpr int kAxesLds = 2048;      // axes up to this long are summed from LDS
__global__ void __launch_bounds__(kAxesThreads) k_gd_axes(const double* __restrict__ rx, const double* __restrict__ ry,
                                                          int64_t L, int mx, int my, double* gx, double* gy,
                                                          double* ext) {
    AKB_CHAIN_PRIORITY();
    __shared__ double red[4][kAxesThreads / 64];
    double lo_x = INFINITY, hi_x = -INFINITY, lo_y = INFINITY, hi_y = -INFINITY;
    // the ring's points in batches of 16 loads per thread in flight (one memory latency per batch,
    // not one per point)
    for (int64_t r0 = threadIdx.x; r0 < L; r0 += 16 * (int64_t)blockDim.x) {
        double bx[16], by[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int64_t r = r0 + q * (int64_t)blockDim.x;
            bx[q] = r < L ? rx[r] : INFINITY;
            by[q] = r < L ? ry[r] : INFINITY;
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            if (r0 + q * (int64_t)blockDim.x >= L) break;
            lo_x = fmin(lo_x, bx[q]);
            hi_x = fmax(hi_x, bx[q]);
            lo_y = fmin(lo_y, by[q]);
            hi_y = fmax(hi_y, by[q]);
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        lo_x = fmin(lo_x, __shfl_down(lo_x, off));
        hi_x = fmax(hi_x, __shfl_down(hi_x, off));
        lo_y = fmin(lo_y, __shfl_down(lo_y, off));
        hi_y = fmax(hi_y, __shfl_down(hi_y, off));
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = lo_x;
        red[1][threadIdx.x >> 6] = hi_x;
        red[2][threadIdx.x >> 6] = lo_y;
        red[3][threadIdx.x >> 6] = hi_y;
    }
    __syncthreads();
    double e[4];
    for (int q = 0; q < 4; ++q) {
        e[q] = red[q][0];
        for (int w = 1; w < kAxesThreads / 64; ++w) e[q] = (q & 1) ? fmax(e[q], red[q][w]) : fmin(e[q], red[q][w]);
    }
    if (threadIdx.x == 0 && ext)
        for (int q = 0; q < 4; ++q) ext[q] = e[q];
    // the axes also into LDS (when they fit) for the pitch's meshgrid sums below
    __shared__ double sgx[kAxesLds], sgy[kAxesLds];
    const bool lds = mx <= kAxesLds && my <= kAxesLds;
    auto lin = [&](double a0, double a1, int m, double* out, double* sout) {
        if (m == 1) {
            if (threadIdx.x == 0) {
                out[0] = a0;
                if (lds) sout[0] = a0;
            }
            return;
        }
        const double step = (a1 - a0) / (double)(m - 1);
        for (int i = threadIdx.x; i < m; i += blockDim.x) {
            double v;
            if (step == 0) v = (double)i / (double)(m - 1) * (a1 - a0) + a0;  // numpy's zero-step branch
            else v = (double)i * step + a0;
            out[i] = i == m - 1 ? a1 : v;
            if (lds) sout[i] = i == m - 1 ? a1 : v;
        }
    };
    lin(e[0], e[1], mx, gx, sgx);
    lin(e[2], e[3], my, gy, sgy);
    if (!ext) return;
    // the pupil pitch psf_calc takes after the driver's grid_H -= np.mean(grid_H) (:3698, :1176-1177):
    // dx = |gh[0,1] - gh[0,0]|, dy = |gv[1,0] - gv[0,0]| of the mean-subtracted meshgrids, each mean
    // numpy's (pairwise over the flattened my x mx meshgrid), waves 0 and 1
    __shared__ PwTree tree[2];
    __threadfence_block();
    __syncthreads();  // the axes are written
    const int w = threadIdx.x >> 6;
    if (w < 2) {
        const long long cnt = (long long)mx * my;
        const double* a = lds ? (w == 0 ? sgx : sgy) : (w == 0 ? gx : gy);
        const int m = w == 0 ? mx : my;
        double sum;
        sum = pw_sum_wave_get(tree[w], MeshgridAxis{a, mx, w == 0}, cnt);
        const double mean = sum / (double)cnt;
        if ((threadIdx.x & 63) == 0) ext[4 + w] = m > 1 ? fabs((a[1] - mean) - (a[0] - mean)) : 0.0;
    }
}

// whether triangle o lies in an interior target cell (a patch's: its (2K + 4)^2 box clear of the
// ring by one vertex), and that cell and its p00 vertex; else the boundary band forms its corners
__device__ __forceinline__ bool cone_interior(const Grid& g, int o, int K, int64_t& c, int64_t& p00) {
    if (o >= 2 * ncells(g)) return false;
    c = o >> 1;
    const int iv = (int)(c / (g.nh - 1)), ih = (int)(c - (int64_t)iv * (g.nh - 1));
    p00 = (int64_t)iv * g.nh + ih;
    return iv - K - 1 >= 1 && iv + K + 2 <= g.nv - 2 && ih - K - 1 >= 1 && ih + K + 2 <= g.nh - 2;
}

// a sharded lattice's targets: this rank forms the interior targets whose cell's p00 lies in its
// rays [own0, own1); the band owner forms every band and pocket target. assigned[t] = 1 for the
// targets formed here; the interior ones' cells go to the patch list
__global__ void __launch_bounds__(kBlock) k_gd_cone_assign(Grid g, const int* __restrict__ owner, int64_t m, int K,
                                                            int64_t own0, int64_t own1, int band_on, int64_t* cells,
                                                            int* count, int* band, uint8_t* assigned) {
    AKB_CHAIN_PRIORITY();
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < m; t += (int64_t)gridDim.x * blockDim.x) {
        const int o = owner[t];
        uint8_t mine = 0;
        if (o != INT32_MAX) {
            int64_t c = -1, p00 = -1;
            const bool interior = cone_interior(g, o, K, c, p00);
            if (interior) {
                if (p00 >= own0 && p00 < own1) {
                    cells[atomicAdd(count, 1)] = c;
                    mine = 1;
                }
            } else if (band_on) {
                atomicOr(band, 1);
                mine = 1;
            }
        }
        assigned[t] = mine;
    }
}

// cell triangles (ids < 2 * ncells): one thread each, a box of a few targets
__global__ void __launch_bounds__(kBlock) k_gd_claim(Grid g, Targets t, int* owner) {
    AKB_CHAIN_PRIORITY();
    const int64_t ntri = 2 * ncells(g);
    for (int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; id < ntri; id += (int64_t)gridDim.x * blockDim.x) {
        const Tri T = tri_verts(g, id);
        int c0, c1, r0, r1;
        tri_box(g, t, T, c0, c1, r0, r1);
        for (int r = r0; r < r1; ++r)
            for (int c = c0; c < c1; ++c) claim_one(g, t, T, (int)id, r, c, owner);
    }
}

// cell triangles, one thread per cell: the targets are sparse against the cells (a 128^2 pupil
// grid over 1e7 hits), so the cell's target index box is first estimated from the linspace axes
// (widened by one index each way) and almost every thread stops there; the candidates are then
// held to each triangle's exact box and barycentric test, so the claims are k_gd_claim's.
// One cell's claims (its two triangles' targets)
__device__ __forceinline__ void claim_cell(const Grid& g, const Targets& t, int64_t c, bool uniform, double inv_dx,
                                           double inv_dy, int* owner) {
    const int iv = (int)(c / (g.nh - 1)), ih = (int)(c - (int64_t)iv * (g.nh - 1));
    const int64_t p00 = (int64_t)iv * g.nh + ih;
    const double xa = g.x[p00], xb = g.x[p00 + 1], xc = g.x[p00 + g.nh], xd = g.x[p00 + g.nh + 1];
    const double ya = g.y[p00], yb = g.y[p00 + 1], yc = g.y[p00 + g.nh], yd = g.y[p00 + g.nh + 1];
    const double xlo = fmin(fmin(xa, xb), fmin(xc, xd)), xhi = fmax(fmax(xa, xb), fmax(xc, xd));
    const double ylo = fmin(fmin(ya, yb), fmin(yc, yd)), yhi = fmax(fmax(ya, yb), fmax(yc, yd));
    const double padx = (xhi - xlo) * 1e-9, pady = (yhi - ylo) * 1e-9;
    int c0, c1, r0, r1;
    if (uniform) {
        if (!axis_range(t.gx, t.mx, inv_dx, xlo - padx, xhi + padx, c0, c1)) return;
        if (!axis_range(t.gy, t.my, inv_dy, ylo - pady, yhi + pady, r0, r1)) return;
    } else {
        c0 = lower_idx(t.gx, t.mx, xlo - padx);
        c1 = lower_idx(t.gx, t.mx, xhi + padx);
        r0 = lower_idx(t.gy, t.my, ylo - pady);
        r1 = lower_idx(t.gy, t.my, yhi + pady);
        if (c0 >= c1 || r0 >= r1) return;
    }
    // the exact box within the estimate: targets with lo <= coordinate < hi (as lower_idx gives)
    while (c0 < c1 && t.gx[c0] < xlo - padx) ++c0;
    while (c1 > c0 && t.gx[c1 - 1] >= xhi + padx) --c1;
    if (c0 >= c1) return;
    while (r0 < r1 && t.gy[r0] < ylo - pady) ++r0;
    while (r1 > r0 && t.gy[r1 - 1] >= yhi + pady) --r1;
    if (r0 >= r1) return;
    for (int half = 0; half < 2; ++half) {
        const int64_t id = 2 * c + half;
        const Tri T = tri_verts(g, id);
        // tri_box within the cell's box: the triangle's padded range lies inside the cell's, so its
        // lower_idx bounds lie in [c0, c1] / [r0, r1] and a scan from the cell's bounds finds them
        // (the binary searches over the whole axis were the kernel's longest dependent chains)
        double txlo = g.x[T.v[0]], txhi = txlo, tylo = g.y[T.v[0]], tyhi = tylo;
        for (int k = 1; k < 3; ++k) {
            txlo = fmin(txlo, g.x[T.v[k]]);
            txhi = fmax(txhi, g.x[T.v[k]]);
            tylo = fmin(tylo, g.y[T.v[k]]);
            tyhi = fmax(tyhi, g.y[T.v[k]]);
        }
        const double tpx = (txhi - txlo) * 1e-9, tpy = (tyhi - tylo) * 1e-9;
        int tc0 = c0, tr0 = r0;
        while (tc0 < c1 && t.gx[tc0] < txlo - tpx) ++tc0;
        int tc1 = tc0;
        while (tc1 < c1 && t.gx[tc1] < txhi + tpx) ++tc1;
        while (tr0 < r1 && t.gy[tr0] < tylo - tpy) ++tr0;
        int tr1 = tr0;
        while (tr1 < r1 && t.gy[tr1] < tyhi + tpy) ++tr1;
        for (int r = tr0; r < tr1; ++r)
            for (int cc = tc0; cc < tc1; ++cc) claim_one(g, t, T, (int)id, r, cc, owner);
    }
}

__global__ void __launch_bounds__(kBlock) k_gd_claim_cells(Grid g, Targets t, int* owner) {
    AKB_CHAIN_PRIORITY();
    const bool uniform = axes_uniform(t);
    const double inv_dx = inv_step(t.gx, t.mx), inv_dy = inv_step(t.gy, t.my);
    for (int64_t c = win_cell0(g) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < win_cell1(g);
         c += (int64_t)gridDim.x * blockDim.x)
        claim_cell(g, t, c, uniform, inv_dx, inv_dy, owner);
}

// k_gd_claim_cells by 8 x 8 blocks of the window's cells, a wave each: the bounding box of the
// block's 9 x 9 vertices (a superset of each of its cells' boxes, so of their candidate targets)
// tested first, and only a block with a candidate target claims cell by cell. The targets are
// sparse against the cells (a 128^2 grid over 1e7 cells: ~85 % of the blocks hold none), so most
// cells are settled by one 81-vertex load per block. Same claims as k_gd_claim_cells.
__global__ void __launch_bounds__(kBlock) k_gd_claim_blocks(Grid g, Targets t, int* owner) {
    AKB_CHAIN_PRIORITY();
    const bool uniform = axes_uniform(t);
    const double inv_dx = inv_step(t.gx, t.mx), inv_dy = inv_step(t.gy, t.my);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int r_lo = g.row0, r_hi = g.row1 < 0 ? g.nv - 1 : g.row1;
    const int bh = (g.nh - 1 + 7) / 8;
    const int64_t nblk = (int64_t)((r_hi - r_lo + 7) / 8) * bh;
    for (int64_t blk = (int64_t)blockIdx.x * nw + wv; blk < nblk; blk += (int64_t)gridDim.x * nw) {
        const int bv = (int)(blk / bh), bc = (int)(blk - (int64_t)bv * bh);
        const int iv0 = r_lo + bv * 8, ih0 = bc * 8;
        const int nr = min(8, r_hi - iv0), nc = min(8, g.nh - 1 - ih0);  // cells; vertices one more
        double xlo = INFINITY, xhi = -INFINITY, ylo = INFINITY, yhi = -INFINITY;
        bool nonfinite = false;
        for (int k = lane; k < (nr + 1) * (nc + 1); k += 64) {
            const int vr = k / (nc + 1), vc = k - (k / (nc + 1)) * (nc + 1);
            const int64_t q = (int64_t)(iv0 + vr) * g.nh + (ih0 + vc);
            const double x = g.x[q], y = g.y[q];
            nonfinite = nonfinite || !isfinite(x) || !isfinite(y);
            xlo = fmin(xlo, x);
            xhi = fmax(xhi, x);
            ylo = fmin(ylo, y);
            yhi = fmax(yhi, y);
        }
        for (int off = 32; off > 0; off >>= 1) {
            xlo = fmin(xlo, __shfl_xor(xlo, off));
            xhi = fmax(xhi, __shfl_xor(xhi, off));
            ylo = fmin(ylo, __shfl_xor(ylo, off));
            yhi = fmax(yhi, __shfl_xor(yhi, off));
        }
        // a non-finite vertex (a run that raises): its cells as k_gd_claim_cells would see them
        const bool any_nf = __any(nonfinite);
        if (!any_nf) {
            const double padx = (xhi - xlo) * 1e-9, pady = (yhi - ylo) * 1e-9;
            int c0, c1, r0, r1;
            bool hit;
            if (uniform) {
                hit = axis_range(t.gx, t.mx, inv_dx, xlo - padx, xhi + padx, c0, c1) &&
                      axis_range(t.gy, t.my, inv_dy, ylo - pady, yhi + pady, r0, r1);
            } else {
                hit = lower_idx(t.gx, t.mx, xlo - padx) < lower_idx(t.gx, t.mx, xhi + padx) &&
                      lower_idx(t.gy, t.my, ylo - pady) < lower_idx(t.gy, t.my, yhi + pady);
            }
            if (!hit) continue;
        }
        const int rr = lane >> 3, cc = lane & 7;
        if (rr < nr && cc < nc) claim_cell(g, t, (int64_t)(iv0 + rr) * (g.nh - 1) + (ih0 + cc), uniform, inv_dx, inv_dy,
                                           owner);
    }
}

// The claims in two launches (the cone solve's, with scratch): k_gd_claim_scan - one thread per
// 8 x 8 block of the window's cells, the bounding box of its 9 x 9 vertices tested against the
// target axes (a superset of its cells' candidate targets; a non-finite vertex marks the block) -
// then k_gd_claim_hit, a wave per marked block claiming cell by cell. The scan holds few registers,
// so the whole GPU's worth of blocks is in flight at once (k_gd_claim_blocks' waves, sized for the
// per-cell claims, walk ~40 blocks each, one load latency after another). Same claims.
__device__ __forceinline__ void claim_block_dims(const Grid& g, int64_t& nblk, int& bh, int& r_lo, int& r_hi) {
    r_lo = g.row0;
    r_hi = g.row1 < 0 ? g.nv - 1 : g.row1;
    bh = (g.nh - 1 + 7) / 8;
    nblk = (int64_t)((r_hi - r_lo + 7) / 8) * bh;
}

__global__ void __launch_bounds__(kBlock) k_gd_claim_scan(Grid g, Targets t, uint8_t* hit) {
    AKB_CHAIN_PRIORITY();
    const bool uniform = axes_uniform(t);
    const double inv_dx = inv_step(t.gx, t.mx), inv_dy = inv_step(t.gy, t.my);
    int64_t nblk;
    int bh, r_lo, r_hi;
    claim_block_dims(g, nblk, bh, r_lo, r_hi);
    for (int64_t blk = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; blk < nblk;
         blk += (int64_t)gridDim.x * blockDim.x) {
        const int bv = (int)(blk / bh), bc = (int)(blk - (int64_t)bv * bh);
        const int iv0 = r_lo + bv * 8, ih0 = bc * 8;
        const int nr = min(8, r_hi - iv0), nc = min(8, g.nh - 1 - ih0);
        // the block's extent from its boundary vertices only (32 of 81): on an unfolded lattice of
        // convex cells an interior vertex lies inside the union of its cells, so no extreme is its
        // alone - the same box as over all 81. (A folded lattice or a non-finite hit fails the run
        // from the cell pass's flags; its claims are never used.)
        double xlo = INFINITY, xhi = -INFINITY, ylo = INFINITY, yhi = -INFINITY;
        bool nonfinite = false;
        auto take = [&](int64_t q) {
            const double x = g.x[q], y = g.y[q];
            nonfinite = nonfinite || !isfinite(x) || !isfinite(y);
            xlo = fmin(xlo, x);
            xhi = fmax(xhi, x);
            ylo = fmin(ylo, y);
            yhi = fmax(yhi, y);
        };
        for (int vr = 0; vr <= nr; ++vr) {
            const int64_t q0 = (int64_t)(iv0 + vr) * g.nh + ih0;
            if (vr == 0 || vr == nr) {
                for (int vc = 0; vc <= nc; ++vc) take(q0 + vc);
            } else {
                take(q0);
                take(q0 + nc);
            }
        }
        bool h = nonfinite;
        if (!h) {
            const double padx = (xhi - xlo) * 1e-9, pady = (yhi - ylo) * 1e-9;
            int c0, c1, r0, r1;
            if (uniform) {
                h = axis_range(t.gx, t.mx, inv_dx, xlo - padx, xhi + padx, c0, c1) &&
                    axis_range(t.gy, t.my, inv_dy, ylo - pady, yhi + pady, r0, r1);
            } else {
                h = lower_idx(t.gx, t.mx, xlo - padx) < lower_idx(t.gx, t.mx, xhi + padx) &&
                    lower_idx(t.gy, t.my, ylo - pady) < lower_idx(t.gy, t.my, yhi + pady);
            }
        }
        hit[blk] = h ? 1 : 0;
    }
}

__global__ void __launch_bounds__(kBlock, 5) k_gd_claim_hit(Grid g, Targets t, const uint8_t* __restrict__ hit,
                                                         int* owner) {
    AKB_CHAIN_PRIORITY();
    const bool uniform = axes_uniform(t);
    const double inv_dx = inv_step(t.gx, t.mx), inv_dy = inv_step(t.gy, t.my);
    // the target axes in LDS: the claims' index scans walk them one dependent load at a time
    __shared__ double sax[2 * kClaimAxisLds];
    Targets tl = t;
    if (t.mx <= kClaimAxisLds && t.my <= kClaimAxisLds) {
        for (int i = threadIdx.x; i < t.mx; i += blockDim.x) sax[i] = t.gx[i];
        for (int i = threadIdx.x; i < t.my; i += blockDim.x) sax[kClaimAxisLds + i] = t.gy[i];
        __syncthreads();
        tl.gx = sax;
        tl.gy = sax + kClaimAxisLds;
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    int64_t nblk;
    int bh, r_lo, r_hi;
    claim_block_dims(g, nblk, bh, r_lo, r_hi);
    for (int64_t blk = (int64_t)blockIdx.x * nw + wv; blk < nblk; blk += (int64_t)gridDim.x * nw) {
        if (!hit[blk]) continue;
        const int bv = (int)(blk / bh), bc = (int)(blk - (int64_t)bv * bh);
        const int iv0 = r_lo + bv * 8, ih0 = bc * 8;
        const int nr = min(8, r_hi - iv0), nc = min(8, g.nh - 1 - ih0);
        const int rr = lane >> 3, cc = lane & 7;
        if (rr < nr && cc < nc) claim_cell(g, tl, (int64_t)(iv0 + rr) * (g.nh - 1) + (ih0 + cc), uniform, inv_dx, inv_dy,
                                           owner);
    }
}

// pocket triangles: slivers along the boundary whose boxes hold from none to thousands of targets,
// so one wave per triangle, its lanes striding the box (a workgroup per triangle left most of its
// threads idle on the common few-target boxes; a thread per triangle left the long slivers' boxes
// to one lane each: 326 us against 28 at C3); the target axes in LDS for tri_box's binary searches
__global__ void __launch_bounds__(kBlock) k_gd_claim_pockets(Grid g, Targets t, int* owner) {
    AKB_CHAIN_PRIORITY();
    const int64_t nc2 = 2 * ncells(g);
    const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    __shared__ double sax[2 * kClaimAxisLds];
    if (t.mx <= kClaimAxisLds && t.my <= kClaimAxisLds) {
        for (int i = threadIdx.x; i < t.mx; i += blockDim.x) sax[i] = t.gx[i];
        for (int i = threadIdx.x; i < t.my; i += blockDim.x) sax[kClaimAxisLds + i] = t.gy[i];
        __syncthreads();
        t.gx = sax;
        t.gy = sax + kClaimAxisLds;
    }
    for (int64_t j = (int64_t)blockIdx.x * nw + (threadIdx.x >> 6); j < g.npock; j += (int64_t)gridDim.x * nw) {
        const Tri T = tri_verts(g, nc2 + j);
        int c0, c1, r0, r1;
        tri_box(g, t, T, c0, c1, r0, r1);
        const int w = c1 - c0;
        const int64_t m = (int64_t)w * (r1 - r0);
        for (int64_t k = lane; k < m; k += 64) {
            const int r = r0 + (int)(k / w), c = c0 + (int)(k - (int64_t)(k / w) * w);
            claim_one(g, t, T, (int)(nc2 + j), r, c, owner);
        }
    }
}

// the values clough_tocher reads for a triangle: its vertices' positions, f and gradients, and its
// three neighbour triangles' centroids (nb false: a hull edge)
struct CTIn {
    double px[3], py[3], f[3], gx[3], gy[3];
    double cx[3], cy[3];
    bool nb[3];
};

// bary's arithmetic on the triangle's vertex values
__device__ __forceinline__ void bary_v(const double (&x)[3], const double (&y)[3], double px, double py,
                                       double (&b)[3]) {
    const double x2 = x[2], y2 = y[2];
    const double a00 = x[0] - x2, a01 = x[1] - x2;
    const double a10 = y[0] - y2, a11 = y[1] - y2;
    const double det = a00 * a11 - a01 * a10;
    const double t00 = a11 / det, t01 = -a01 / det, t10 = -a10 / det, t11 = a00 / det;
    const double dx = px - x2, dy = py - y2;
    b[0] = t00 * dx + t01 * dy;
    b[1] = t10 * dx + t11 * dy;
    b[2] = 1.0 - b[0] - b[1];
}

// scipy's Clough-Tocher patch at barycentric b from the gathered values
__device__ double ct_eval(const CTIn& in, const double (&b)[3]) {
    const double p0x = in.px[0], p0y = in.py[0];
    const double p1x = in.px[1], p1y = in.py[1];
    const double p2x = in.px[2], p2y = in.py[2];
    const double e12x = p1x - p0x, e12y = p1y - p0y;
    const double e23x = p2x - p1x, e23y = p2y - p1y;
    const double e31x = p0x - p2x, e31y = p0y - p2y;
    const double f1 = in.f[0], f2 = in.f[1], f3 = in.f[2];
    const double g0x = in.gx[0], g0y = in.gy[0];
    const double g1x = in.gx[1], g1y = in.gy[1];
    const double g2x = in.gx[2], g2y = in.gy[2];
    const double df12 = +(g0x * e12x + g0y * e12y);
    const double df21 = -(g1x * e12x + g1y * e12y);
    const double df23 = +(g1x * e23x + g1y * e23y);
    const double df32 = -(g2x * e23x + g2y * e23y);
    const double df31 = +(g2x * e31x + g2y * e31y);
    const double df13 = -(g0x * e31x + g0y * e31y);
    const double c3000 = f1, c2100 = (df12 + 3 * c3000) / 3, c2010 = (df13 + 3 * c3000) / 3;
    const double c0300 = f2, c1200 = (df21 + 3 * c0300) / 3, c0210 = (df23 + 3 * c0300) / 3;
    const double c0030 = f3, c1020 = (df31 + 3 * c0030) / 3, c0120 = (df32 + 3 * c0030) / 3;
    const double c2001 = (c2100 + c2010 + c3000) / 3;
    const double c0201 = (c1200 + c0300 + c0210) / 3;
    const double c0021 = (c1020 + c0120 + c0030) / 3;
    double gk[3];
    for (int k = 0; k < 3; ++k) {
        if (!in.nb[k]) {
            gk[k] = -0.5;
            continue;
        }
        double c[3];
        bary_v(in.px, in.py, in.cx[k], in.cy[k], c);
        if (k == 0) gk[k] = (2 * c[2] + c[1] - 1) / (2 - 3 * c[2] - 3 * c[1]);
        else if (k == 1) gk[k] = (2 * c[0] + c[2] - 1) / (2 - 3 * c[0] - 3 * c[2]);
        else gk[k] = (2 * c[1] + c[0] - 1) / (2 - 3 * c[1] - 3 * c[0]);
    }
    const double c0111 = (gk[0] * (-c0300 + 3 * c0210 - 3 * c0120 + c0030) + (-c0300 + 2 * c0210 - c0120 + c0021 + c0201)) / 2;
    const double c1011 = (gk[1] * (-c0030 + 3 * c1020 - 3 * c2010 + c3000) + (-c0030 + 2 * c1020 - c2010 + c2001 + c0021)) / 2;
    const double c1101 = (gk[2] * (-c3000 + 3 * c2100 - 3 * c1200 + c0300) + (-c3000 + 2 * c2100 - c1200 + c2001 + c0201)) / 2;
    const double c1002 = (c1101 + c1011 + c2001) / 3;
    const double c0102 = (c1101 + c0111 + c0201) / 3;
    const double c0012 = (c1011 + c0111 + c0021) / 3;
    const double c0003 = (c1002 + c0102 + c0012) / 3;
    const double mv = fmin(b[0], fmin(b[1], b[2]));
    const double b1 = b[0] - mv, b2 = b[1] - mv, b3 = b[2] - mv, b4 = 3 * mv;
    return b1 * b1 * b1 * c3000 + 3 * b1 * b1 * b2 * c2100 + 3 * b1 * b1 * b3 * c2010 + 3 * b1 * b1 * b4 * c2001 +
           3 * b1 * b2 * b2 * c1200 + 6 * b1 * b2 * b4 * c1101 + 3 * b1 * b3 * b3 * c1020 + 6 * b1 * b3 * b4 * c1011 +
           3 * b1 * b4 * b4 * c1002 + b2 * b2 * b2 * c0300 + 3 * b2 * b2 * b3 * c0210 + 3 * b2 * b2 * b4 * c0201 +
           3 * b2 * b3 * b3 * c0120 + 6 * b2 * b3 * b4 * c0111 + 3 * b2 * b4 * b4 * c0102 + b3 * b3 * b3 * c0030 +
           3 * b3 * b3 * b4 * c0021 + 3 * b3 * b4 * b4 * c0012 + b4 * b4 * b4 * c0003;
}


// the generic gather (any triangle: lattice cells at the boundary, pockets) through tri_nbr / tri_verts
__device__ void ct_gather(const Grid& g, int64_t tid, const Tri& T, const double* f, const double* grad, CTIn& in) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        in.px[k] = g.x[T.v[k]];
        in.py[k] = g.y[T.v[k]];
        in.f[k] = f[T.v[k]];
        in.gx[k] = grad[2 * T.v[k]];
        in.gy[k] = grad[2 * T.v[k] + 1];
    }
    for (int k = 0; k < 3; ++k) {
        const int64_t n = tri_nbr(g, tid, k);
        in.nb[k] = n >= 0;
        if (n < 0) continue;
        const Tri N = tri_verts(g, n);
        in.cx[k] = (g.x[N.v[0]] + g.x[N.v[1]] + g.x[N.v[2]]) / 3;
        in.cy[k] = (g.y[N.v[0]] + g.y[N.v[1]] + g.y[N.v[2]]) / 3;
    }
}

__device__ double clough_tocher(const Grid& g, int64_t tid, const Tri& T, const double* f, const double* grad,
                                const double (&b)[3]) {
    CTIn in;
    ct_gather(g, tid, T, f, grad, in);
    return ct_eval(in, b);
}

// a cell triangle's vertices (tri_verts' order) from its cell's first corner, diagonal and half
__device__ __forceinline__ void cell_tri(int64_t p00, int64_t nh, int d, int half, int64_t (&v)[3]) {
    const int64_t p01 = p00 + 1, p10 = p00 + nh, p11 = p10 + 1;
    if (d == 0) {
        v[0] = p00;
        v[1] = half == 0 ? p01 : p11;
        v[2] = half == 0 ? p11 : p10;
    } else {
        v[0] = half == 0 ? p00 : p01;
        v[1] = half == 0 ? p01 : p11;
        v[2] = p10;
    }
}

// ct_gather for a lattice triangle whose cell is one cell clear of the ring (its four neighbour
// cells are lattice cells, so tri_nbr takes no ring edge or pocket): the five cells' diagonals in
// one batch, then every vertex value - the triangle's and its neighbours' - in a second, instead of
// tri_verts -> tri_nbr -> across_side -> tri_verts one dependent load after another. The same
// triangles and the same values, so ct_eval gives clough_tocher's bits. y2 (or nullptr): a second
// gradient set (the band's extra sweep) into gy2x / gy2y. false: not such a triangle.
__device__ __forceinline__ bool ct_gather_lattice(const Grid& g, int o, const double* f, const double* grad,
                                                  const double* y2, CTIn& in, double (&g2x)[3], double (&g2y)[3],
                                                  Tri& T) {
    const int64_t nc2 = 2 * ncells(g);
    if (o >= nc2) return false;
    const int64_t c = o >> 1;
    const int half = o & 1;
    const int64_t w = g.nh - 1;
    const int iv = (int)(c / w), ih = (int)(c - (int64_t)iv * w);
    if (iv < 1 || iv > g.nv - 3 || ih < 1 || ih > g.nh - 3) return false;
    const int d = g.diag[c], dB = g.diag[c - w], dT = g.diag[c + w], dL = g.diag[c - 1], dR = g.diag[c + 1];
    const int64_t p00 = (int64_t)iv * g.nh + ih;
    cell_tri(p00, g.nh, d, half, T.v);
    // the neighbour across the side opposite vertex k (tri_nbr's table and across_side's cells)
    constexpr uint64_t kSide = (2ull << 0) | (0ull << 3) | (1ull << 6) | (3ull << 9) | (4ull << 12) | (0ull << 15) |
                               (0ull << 18) | (4ull << 21) | (1ull << 24) | (3ull << 27) | (0ull << 30) | (2ull << 33);
    int64_t nv_[3][3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int side = (int)((kSide >> (3 * ((d * 2 + half) * 3 + k))) & 7u) - 1;
        if (side < 0) cell_tri(p00, g.nh, d, 1 - half, nv_[k]);                    // the cell's other half
        else if (side == 0) cell_tri(p00 - g.nh, g.nh, dB, 1, nv_[k]);             // below: its top edge
        else if (side == 2) cell_tri(p00 + g.nh, g.nh, dT, 0, nv_[k]);             // above: its bottom edge
        else if (side == 1) cell_tri(p00 + 1, g.nh, dR, dR == 0 ? 1 : 0, nv_[k]);  // right: its left edge
        else cell_tri(p00 - 1, g.nh, dL, dL == 0 ? 0 : 1, nv_[k]);                 // left: its right edge
    }
    double nx[3][3], ny[3][3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        in.px[k] = g.x[T.v[k]];
        in.py[k] = g.y[T.v[k]];
        in.f[k] = f[T.v[k]];
        in.gx[k] = grad[2 * T.v[k]];
        in.gy[k] = grad[2 * T.v[k] + 1];
        g2x[k] = y2 ? y2[2 * T.v[k]] : 0.0;
        g2y[k] = y2 ? y2[2 * T.v[k] + 1] : 0.0;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            nx[k][q] = g.x[nv_[k][q]];
            ny[k][q] = g.y[nv_[k][q]];
        }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        in.nb[k] = true;
        in.cx[k] = (nx[k][0] + nx[k][1] + nx[k][2]) / 3;
        in.cy[k] = (ny[k][0] + ny[k][1] + ny[k][2]) / 3;
    }
    return true;
}

// nvals value sets share the triangulation: f / grad / out strided by n / 2n / mx*my
// The cone solve's estimates at the band's targets (be.y != nullptr: the band's one more plain
// sweep y from x_K), for each target whose triangle is not an interior cell's - the boundary
// cells' and the pocket triangles': the change measure of that sweep at the triangle's vertices
// and, as the value-error estimate, twice the value change it makes at the target (the
// Clough-Tocher value is linear in the gradients and the fixed point lies within ~2x the Jacobi
// step; a pocket sliver's long edges carry the step furthest, so its value, not a bound through
// the edge length, is taken), as ordered double bits
struct BandEst {
    const double* y;  // (n, 2) or nullptr
    int K;
    unsigned long long* chg;
    unsigned long long* est;
};

__device__ __forceinline__ void band_target_est(const Grid& g, const BandEst& be, int o, const Tri& T,
                                                const double* f, const double* grad, const double (&b)[3], double v0,
                                                double& cmax, double& emax) {
    int64_t c, p00;
    if (cone_interior(g, o, be.K, c, p00)) return;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int64_t v = T.v[k];
        cmax = fmax(cmax, change_of(grad[2 * v], grad[2 * v + 1], be.y[2 * v], be.y[2 * v + 1]));
    }
    emax = nan_max(emax, 2.0 * fabs(clough_tocher(g, o, T, f, be.y, b) - v0));  // (a NaN kept: refused)
}

__device__ __forceinline__ void band_est_store(const BandEst& be, double cmax, double emax) {
    for (int off = 32; off > 0; off >>= 1) {
        cmax = fmax(cmax, __shfl_down(cmax, off));
        emax = nan_max(emax, __shfl_down(emax, off));
    }
    if ((threadIdx.x & 63) == 0) {
        if (be.chg && cmax > 0) atomicMax(be.chg, (unsigned long long)__double_as_longlong(cmax));
        // a NaN estimate (a non-finite value at a band target) as +inf: above any bar
        if (be.est && (emax > 0 || emax != emax))
            atomicMax(be.est, (unsigned long long)__double_as_longlong(emax != emax ? HUGE_VAL : emax));
    }
}

__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) k_gd_eval(Grid g, Targets t, const int* __restrict__ owner,
                                                    const double* f, const double* grad, int nvals, double* out,
                                                    BandEst be = BandEst{nullptr, 0, nullptr, nullptr}) {
    AKB_CHAIN_PRIORITY();
    const int64_t m = (int64_t)t.mx * t.my, n = (int64_t)g.nv * g.nh;
    double cmax = 0.0, emax = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const int o = owner[i];
        if (o == INT32_MAX) {
            for (int v = 0; v < nvals; ++v) out[v * m + i] = __builtin_nan("");
            continue;
        }
        const int r = (int)(i / t.mx), c = (int)(i - (int64_t)r * t.mx);
        if (nvals == 1) {  // the cone solve's: the batched gather where it applies
            CTIn in;
            double g2x[3], g2y[3];
            Tri T;
            if (ct_gather_lattice(g, o, f, grad, be.y, in, g2x, g2y, T)) {
                double b[3];
                bary_v(in.px, in.py, t.gx[c], t.gy[r], b);
                const double v0 = ct_eval(in, b);
                out[i] = v0;
                int64_t cc, p00;
                if (be.y && !cone_interior(g, o, be.K, cc, p00)) {  // band_target_est on the gathered values
#pragma unroll
                    for (int k = 0; k < 3; ++k) cmax = fmax(cmax, change_of(in.gx[k], in.gy[k], g2x[k], g2y[k]));
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        in.gx[k] = g2x[k];
                        in.gy[k] = g2y[k];
                    }
                    emax = nan_max(emax, 2.0 * fabs(ct_eval(in, b) - v0));
                }
                continue;
            }
        }
        const Tri T = tri_verts(g, o);
        double b[3];
        bary(g, T, t.gx[c], t.gy[r], b);
        for (int v = 0; v < nvals; ++v) out[v * m + i] = clough_tocher(g, o, T, f + v * n, grad + 2 * v * n, b);
        if (be.y) band_target_est(g, be, o, T, f, grad, b, out[i], cmax, emax);  // (one value set)
    }
    if (be.y) band_est_store(be, cmax, emax);
}

// k_gd_eval for the targets a rank forms (assigned): value and count, zeros elsewhere, so the
// ranks' pieces add up to the map (a SUM reduction; count 0: outside the hull, NaN)
__global__ void __launch_bounds__(kBlock) k_gd_eval_part(Grid g, Targets t, const int* __restrict__ owner,
                                                         const uint8_t* __restrict__ assigned, const double* f,
                                                         const double* grad, int nvals, double* out, double* cnt,
                                                         BandEst be = BandEst{nullptr, 0, nullptr, nullptr}) {
    AKB_CHAIN_PRIORITY();
    const int64_t m = (int64_t)t.mx * t.my, n = (int64_t)g.nv * g.nh;
    double cmax = 0.0, emax = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        if (!assigned[i]) {
            for (int v = 0; v < nvals; ++v) out[v * m + i] = 0.0;
            cnt[i] = 0.0;
            continue;
        }
        const int o = owner[i];
        const int r = (int)(i / t.mx), c = (int)(i - (int64_t)r * t.mx);
        const Tri T = tri_verts(g, o);
        double b[3];
        bary(g, T, t.gx[c], t.gy[r], b);
        for (int v = 0; v < nvals; ++v) out[v * m + i] = clough_tocher(g, o, T, f + v * n, grad + 2 * v * n, b);
        cnt[i] = 1.0;
        if (be.y) band_target_est(g, be, o, T, f, grad, b, out[i], cmax, emax);  // (one value set)
    }
    if (be.y) band_est_store(be, cmax, emax);
}

// the assembled pieces: value where some rank formed it, NaN elsewhere (outside the hull)
__global__ void k_gd_part_finish(double* out, const double* cnt, int64_t m, int nvals) {
    AKB_CHAIN_PRIORITY();
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        if (!(cnt[i] > 0))
            for (int v = 0; v < nvals; ++v) out[v * m + i] = __builtin_nan("");
}

__global__ void k_fill_i32(int* p, int64_t n, int v) {
    AKB_CHAIN_PRIORITY();
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

// the strip cell pass's grid for `rows` cell rows of a lattice nh points wide: a wave per strip segment,
// the segments as long as fills the device's wave slots (4 waves per SIMD) once - one round of waves
unsigned gd_cu_count();
struct StripGrid {
    unsigned blocks;
    int seg_rows;
};
StripGrid strip_grid(int nh, int rows) {
    const int64_t nstrip = (nh - 1 + kStripCells - 1) / kStripCells;
    const int64_t slots = (int64_t)gd_cu_count() * 16;
    const int64_t nseg_max = slots / nstrip > 0 ? slots / nstrip : 1;
    const int seg_rows = (int)((rows + nseg_max - 1) / nseg_max) > 8 ? (int)((rows + nseg_max - 1) / nseg_max) : 8;
    const int64_t units = nstrip * ((rows + seg_rows - 1) / seg_rows);
    return StripGrid{(unsigned)((units + kStripThreads / 64 - 1) / (kStripThreads / 64)), seg_rows};
}

// the cell pass over the window's `rows` cell rows
int launch_cells(const Grid& g, uint8_t* diag, double tol, unsigned* d_flags, int rows, hipStream_t s) {
    const StripGrid sg = strip_grid(g.nh, rows);
    k_gd_cells_strip<<<sg.blocks, kStripThreads, 0, s>>>(g, diag, tol, d_flags, sg.seg_rows);
    return launch_status("k_gd_cells");
}
unsigned gd_cu_count() {  // the device's CUs (one resident 1024-thread patch workgroup each)
    static unsigned n = [] {
        int dev = 0, cus = 0;
        return hipGetDevice(&dev) == hipSuccess &&
                       hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0
                   ? (unsigned)cus
                   : 256u;
    }();
    return n;
}
// the per-triangle claim (tests/test_gpu_parity.py's cross-check of the block claims: AKB_GD_CLAIM_TRI)
bool gd_claim_tri() { return getenv("AKB_GD_CLAIM_TRI") != nullptr; }

// diagnostics (akb_gd_patch_timing / akb_gd_patch_times): HIP events around each k_gd_cone_patch
// launch while enabled, a ring of kPatchEvents pairs, and each launch's cell count (its device word)
constexpr int kPatchEvents = 1024;
constexpr int kPatchClk = 10;  // the diagnostics words (akb_gd_patch_phases)
struct PatchTimer {
    bool on = false, made = false;
    bool band_clk = false;  // the band workgroups' clocks too (akb_gd_patch_timing(2): their atomics cost the step)
    hipEvent_t ev[kPatchEvents][2];
    const int* cnt[kPatchEvents];
    hipEvent_t bev[kPatchEvents][2];  // around each value set's band sweeps (the guard's extra sweep included)
    int64_t band_launches = 0;
    int64_t launches = 0;
    unsigned long long* clk = nullptr;  // device: workgroup 0's phase clocks, summed over the launches
};
PatchTimer& patch_timer() {
    static PatchTimer t;
    return t;
}

}  // namespace
}  // namespace akb

using namespace akb;

extern "C" {

// pass 1: cell diagonals + local-Delaunay checks, ring coordinates for the host
int akb_gd_cells_f64(const double* x, const double* y, int nv, int nh, uint8_t* diag, double tol, unsigned* d_flags,
                     double* ring_x, double* ring_y, void* stream) {
    clear_error();
    AKB_REQUIRE(x && y && diag && d_flags && ring_x && ring_y, "null pointer");
    AKB_REQUIRE(nv >= 2 && nh >= 2, "grid of at least 2 x 2 points");
    hipStream_t s = (hipStream_t)stream;
    Grid g{x, y, nv, nh, diag, 0, nullptr, nullptr, nullptr, nullptr, nullptr};
    int st = launch_cells(g, diag, tol, d_flags, nv - 1, s);
    if (st) return st;
    const int64_t L = 2 * (int64_t)(nh - 1) + 2 * (int64_t)(nv - 1);
    k_gd_ring<<<grid_for(L), kBlock, 0, s>>>(g, ring_x, ring_y, d_flags);
    return launch_status("k_gd_ring");
}

int akb_gd_check_pockets(const double* x, const double* y, int nv, int nh, const uint8_t* diag, int npock,
                         const int32_t* ptri, const int32_t* pnbr, const int32_t* edge_tri, double tol,
                         unsigned* d_flags, void* stream) {
    clear_error();
    if (npock == 0) return 0;
    Grid g{x, y, nv, nh, diag, npock, ptri, pnbr, edge_tri, nullptr, nullptr};
    k_gd_check_pockets<<<grid_for(npock), kBlock, 0, (hipStream_t)stream>>>(g, tol, d_flags);
    return launch_status("k_gd_check_pockets");
}

// kk = 1 or 2 Jacobi sweeps in one launch of the register kernel, each a Chebyshev step (om1, om2;
// gprev == NULL: the first is a plain sweep; gin == NULL: x_k = 0). gout1 = x_{k+1}, gout2 =
// x_{k+2}; d_change[0], [1]: the sweeps' largest relative changes; ring_work: 22 L doubles.
int akb_gd_grad_sweeps_f64(const double* x, const double* y, int nv, int nh, const uint8_t* diag, int npock,
                           const int32_t* ptri, const int32_t* pnbr, const int32_t* edge_tri, const int32_t* xptr,
                           const int32_t* xidx, const double* f, int nvals, const double* gin, const double* gprev,
                           double om1, double om2, int kk, double* gout1, double* gout2, double* ring_work,
                           unsigned long long* d_change, void* stream) {
    clear_error();
    AKB_REQUIRE(x && y && diag && f && gout1 && ring_work && d_change && nvals >= 1, "bad arguments");
    AKB_REQUIRE(kk == 1 || (kk == 2 && gout2), "kk must be 1, or 2 with gout2");
    AKB_REQUIRE(!gprev || (om1 > 0 && om1 < 2), "Chebyshev weight outside (0, 2)");
    AKB_REQUIRE(kk == 1 || (om2 > 0 && om2 < 2), "Chebyshev weight outside (0, 2)");
    Grid g{x, y, nv, nh, diag, npock, ptri, pnbr, edge_tri, xptr, xidx};
    const int rows = 24;  // rows per wave: 24 at 3 waves per SIMD measured best on the C3 hits
    hipStream_t s = (hipStream_t)stream;
    const int64_t n = (int64_t)nv * nh;
    const int64_t L = 2 * (int64_t)(nh - 1) + 2 * (int64_t)(nv - 1);
    const unsigned grr = grid_for(L * 64);
    const int own = 64 - 2 * kk;
    const int64_t waves = (int64_t)((nh + own - 1) / own) * ((nv + rows - 1) / rows);
    const unsigned gw = (unsigned)((waves + 3) / 4);
    for (int v = 0; v < nvals; v += 2) {
        const int nv2 = nvals - v >= 2 ? 2 : 1;
        const double* fv = f + v * n;
        const double* gi = gin ? gin + 2 * v * n : nullptr;
        double* o1 = gout1 + 2 * v * n;
        double* o2 = gout2 ? gout2 + 2 * v * n : nullptr;
        double* chords = ring_work;
        double* acc = ring_work + kAccWords(2) * L;
        if (nv2 == 2) {
            k_gd_ring_chords<2><<<grr, kBlock, 0, s>>>(g, fv, gi, chords);
            SweepArgs<2> a{fv, gi, gprev ? gprev + 2 * v * n : nullptr, om1, om2, o1, o2, chords, acc, d_change, rows};
            if (kk == 2) k_gd_sweeps<2, 2, 2><<<gw, 256, 0, s>>>(g, a);  // 180 VGPRs: no spills
            else k_gd_sweeps<2, 1, 1><<<gw, 256, 0, s>>>(g, a);
            if (kk == 2)
                k_gd_grad_ring<2><<<grr, kBlock, 0, s>>>(g, fv, o1, o2, acc, d_change + 1, Cheb{gi, om2, gi ? 0 : 1});
        } else {
            k_gd_ring_chords<1><<<grr, kBlock, 0, s>>>(g, fv, gi, chords);
            SweepArgs<1> a{fv, gi, gprev ? gprev + 2 * v * n : nullptr, om1, om2, o1, o2, chords, acc, d_change, rows};
            if (kk == 2) k_gd_sweeps<1, 2, 1><<<gw, 256, 0, s>>>(g, a);
            else k_gd_sweeps<1, 1, 1><<<gw, 256, 0, s>>>(g, a);
            if (kk == 2)
                k_gd_grad_ring<1><<<grr, kBlock, 0, s>>>(g, fv, o1, o2, acc, d_change + 1, Cheb{gi, om2, gi ? 0 : 1});
        }
        int st = launch_status("k_gd_sweeps");
        if (st) return st;
    }
    return 0;
}

// targets: the meshgrid of gx (mx) x gy (my); owner: (my * mx) int32 scratch; out: (nvals, my, mx)
int akb_gd_eval_f64(const double* x, const double* y, int nv, int nh, const uint8_t* diag, int npock,
                    const int32_t* ptri, const int32_t* pnbr, const int32_t* edge_tri, const double* gx, int mx,
                    const double* gy, int my, const double* f, const double* grad, int nvals, int* owner,
                    double* out, void* stream) {
    clear_error();
    AKB_REQUIRE(x && y && diag && gx && gy && f && grad && owner && out && mx > 0 && my > 0 && nvals >= 1,
                "bad arguments");
    hipStream_t s = (hipStream_t)stream;
    Grid g{x, y, nv, nh, diag, npock, ptri, pnbr, edge_tri, nullptr, nullptr};
    Targets t{gx, gy, mx, my};
    const int64_t m = (int64_t)mx * my;
    k_fill_i32<<<grid_for(m, 4), kBlock, 0, s>>>(owner, m, INT32_MAX);
    int st = launch_status("k_fill_i32");
    if (st) return st;
    const int64_t ntri = 2 * (int64_t)(nv - 1) * (nh - 1) + npock;
    if (gd_claim_tri())  // the per-triangle claim (the tests' cross-check)
        k_gd_claim<<<grid_for(ntri - npock, 1, kStreamGridCap), kBlock, 0, s>>>(g, t, owner);
    else
        k_gd_claim_blocks<<<grid_for((ntri - npock) / 32 + 1, 1, kStreamGridCap), kBlock, 0, s>>>(g, t, owner);
    st = launch_status("k_gd_claim");
    if (st) return st;
    if (npock > 0) {
        const int64_t pw = (npock + kBlock / 64 - 1) / (kBlock / 64);
        k_gd_claim_pockets<<<(unsigned)(pw < 16384 ? pw : 16384), kBlock, 0, s>>>(g, t, owner);
        st = launch_status("k_gd_claim_pockets");
        if (st) return st;
    }
    k_gd_eval<<<grid_for(m, 1, kStreamGridCap), kBlock, 0, s>>>(g, t, owner, f, grad, nvals, out);
    return launch_status("k_gd_eval");
}

int akb_gd_axes_f64(const double* ring_x, const double* ring_y, int64_t L, int mx, int my, double* gx, double* gy,
                    double* d_extent, void* stream) {
    clear_error();
    AKB_REQUIRE(ring_x && ring_y && gx && gy && L > 0 && mx > 0 && my > 0, "bad arguments");
    k_gd_axes<<<1, kAxesThreads, 0, (hipStream_t)stream>>>(ring_x, ring_y, L, mx, my, gx, gy, d_extent);
    return launch_status("k_gd_axes");
}

// ---- cone solve: claims, the fixed-K gradient iteration restricted to what the targets read,
// the patches; one call, no host synchronisation

// the claims' block flags, at the end of the cone work buffer
static int64_t claim_scratch_bytes(int nv, int nh) {
    return ((int64_t)((nv - 1 + 7) / 8) * ((nh - 1 + 7) / 8) + 63) / 64 * 64;
}
static int64_t claim_scratch_offset(int nv, int nh, int mx, int my, int nvals) {
    const int64_t n = (int64_t)nv * nh, L = 2 * (int64_t)(nh - 1) + 2 * (int64_t)(nv - 1);
    const int nv2 = nvals >= 2 ? 2 : 1;
    const int64_t m = (int64_t)mx * my;
    return (3 * (int64_t)nv2 * n * 2 * 8 + L * 16 * 8 + m * 8 + m + 64 + 63) / 64 * 64;
}

int64_t akb_gd_cone_work_bytes(int nv, int nh, int mx, int my, int nvals) {
    if (nv < 2 || nh < 2 || mx < 1 || my < 1 || nvals < 1) return -1;
    return claim_scratch_offset(nv, nh, mx, my, nvals) + claim_scratch_bytes(nv, nh);
}

namespace {

// the cone solve's claims: owner filled with INT32_MAX, then the window's cells (and the pockets)
int cone_claims(const Grid& g, const Targets& t, int with_pockets, int* owner, hipStream_t s, uint8_t* scratch = nullptr) {
    const int64_t m = (int64_t)t.mx * t.my;
    k_fill_i32<<<grid_for(m, 4), kBlock, 0, s>>>(owner, m, INT32_MAX);
    int st = launch_status("k_fill_i32");
    if (st) return st;
    const int64_t wc = (int64_t)((g.row1 < 0 ? g.nv - 1 : g.row1) - g.row0) * (g.nh - 1);
    if (wc > 0) {
        if (scratch) {
            const int64_t nblk = (int64_t)(((g.row1 < 0 ? g.nv - 1 : g.row1) - g.row0 + 7) / 8) * ((g.nh - 1 + 7) / 8);
            k_gd_claim_scan<<<grid_for(nblk, 1, kStreamGridCap), kBlock, 0, s>>>(g, t, scratch);
            if ((st = launch_status("k_gd_claim_scan"))) return st;
            k_gd_claim_hit<<<grid_for(nblk * 16, 1, kStreamGridCap), kBlock, 0, s>>>(g, t, scratch, owner);
        } else {
            k_gd_claim_blocks<<<grid_for(wc / 16 + 1, 1, kStreamGridCap), kBlock, 0, s>>>(g, t, owner);
        }
        if ((st = launch_status("k_gd_claim"))) return st;
    }
    if (with_pockets && g.npock > 0) {
        const int64_t pw = ((int64_t)g.npock + kBlock / 64 - 1) / (kBlock / 64);
        k_gd_claim_pockets<<<(unsigned)(pw < 16384 ? pw : 16384), kBlock, 0, s>>>(g, t, owner);
        if ((st = launch_status("k_gd_claim_pockets"))) return st;
    }
    return 0;
}

// the targets this call forms (own0 .. own1, band_on), their gradients, their values: out / cnt
// as k_gd_eval_part writes them (cnt == nullptr: k_gd_eval's NaN for unclaimed targets). Value sets
// one at a time (a set's iterate does not depend on the others). d_change[0]: the patches' change
// measure, d_change[1]: their value-error estimate (k_gd_cone_patch), ordered double bits.
int cone_part(const Grid& g, const Targets& t, int64_t own0, int64_t own1, int band_on, const double* f, int nvals,
              int K, const double* omegas, void* work, const int* owner, double* out, double* cnt,
              unsigned long long* d_change, hipStream_t s) {
    const int64_t n = (int64_t)g.nv * g.nh, m = (int64_t)t.mx * t.my;
    const int64_t L = 2 * (int64_t)(g.nh - 1) + 2 * (int64_t)(g.nv - 1);
    double* gb[3];
    for (int k = 0; k < 3; ++k) gb[k] = (double*)work + (int64_t)k * n * 2;
    const int nv2 = nvals >= 2 ? 2 : 1;  // the work layout's (claim_scratch_offset)
    int64_t* cells = (int64_t*)((double*)work + 3 * (int64_t)nv2 * n * 2 + L * 16);
    uint8_t* assigned = (uint8_t*)(cells + m);
    int* count = (int*)(((uintptr_t)(assigned + m) + 7) & ~(uintptr_t)7);
    int* band = count + 1;
    if (hipMemsetAsync(count, 0, 2 * sizeof(int), s) != hipSuccess) return launch_status("hipMemsetAsync");
    k_gd_cone_assign<<<grid_for(m, 1), kBlock, 0, s>>>(g, owner, m, K, own0, own1, band_on, cells, count, band,
                                                      assigned);
    int st = launch_status("k_gd_cone_assign");
    if (st) return st;
    // sweep j's form: 1 plain, 2 against x_0 = 0, later against x_{j-2}
    ConeStep steps[kConeMaxK + 1];
    steps[0] = ConeStep{0, 1.0};
    for (int j = 1; j <= K; ++j)
        steps[j] = j == 1 ? ConeStep{0, 1.0} : j == 2 ? ConeStep{1, omegas[1]} : ConeStep{2, omegas[j - 1]};
    // the patches' pipeline split: the smallest S >= K / 2 with the three thread sets (two inner, one
    // outer) and the four corner-store threads in one workgroup
    const int S = patch_split(K);
    const unsigned pp = gd_cu_count();  // one persistent workgroup per CU walks its cells
    AKB_REQUIRE(S >= 0 && m <= 1024 * (int64_t)pp, "cone patches: K or the target count out of range");
    if (patch_order_upload(s)) {
        set_error("cone patches: the vertex order table did not reach constant memory");
        return AKB_E_HIP;
    }
    for (int v = 0; v < nvals; ++v) {
        const double* fv = f + v * n;
        // the boundary band, shrinking like the patches' squares: sweep j forms depth <= 2K + 3 - j,
        // whose neighbours (depth <= 2K + 4 - j) sweep j - 1 formed, so x_K is the global iteration's
        // to depth K + 3 >= every band target's corners (the first sweep reads x_0 = 0 only)
        if (band_on) {
            PatchTimer& bt0 = patch_timer();
            const int bslot = (int)(bt0.band_launches % kPatchEvents);
            if (bt0.on) (void)hipEventRecord(bt0.bev[bslot][0], s);
            // the ring's chord slots (the work's (L, 16)-double region: kChordSlots int32 a vertex)
            int32_t* slots = (int32_t*)((double*)work + 3 * (int64_t)nv2 * n * 2);
            if (v == 0) {
                k_gd_chord_slots<<<grid_for(L), kBlock, 0, s>>>(g, slots, L);
                if ((st = launch_status("k_gd_chord_slots"))) return st;
            }
            for (int j = 1; j <= K; ++j) {
                const double* gin = j == 1 ? nullptr : gb[(j - 1) % 3];
                const double* gprev = j >= 3 ? gb[(j + 1) % 3] : nullptr;
                const BandTiles bt = band_tiles(g.nv, g.nh, 2 * K + 3 - j);
                const ConeBand a{fv, gin, gprev, gb[j % 3], steps[j], band, patch_timer().band_clk ? patch_timer().clk : nullptr,
                                 slots};
                k_gd_cone_band<<<band_grid(bt, L), kBandThreads, 0, s>>>(g, bt, a);
                if ((st = launch_status("k_gd_cone_band"))) return st;
            }
            if (d_change) {  // one more plain sweep, y from x_K to depth K + 2 (the band targets' corners)
                const BandTiles bt = band_tiles(g.nv, g.nh, K + 2);
                const ConeBand a{fv, gb[K % 3], nullptr, gb[(K + 1) % 3], ConeStep{0, 1.0}, band,
                                 patch_timer().band_clk ? patch_timer().clk : nullptr, slots};
                k_gd_cone_band<<<band_grid(bt, L), kBandThreads, 0, s>>>(g, bt, a);
                if ((st = launch_status("k_gd_cone_band"))) return st;
            }
            if (bt0.on) {
                (void)hipEventRecord(bt0.bev[bslot][1], s);
                ++bt0.band_launches;
            }
        }
        const BandEst be{band_on && d_change ? gb[(K + 1) % 3] : nullptr, K, d_change, d_change ? d_change + 1 : nullptr};
        ConePatch a{fv, cells, count, K, {}, gb[K % 3], d_change, d_change ? d_change + 1 : nullptr,
                    patch_timer().on ? patch_timer().clk : nullptr};
        for (int j = 0; j <= K; ++j) a.st[j] = steps[j];
        PatchTimer& pt = patch_timer();
        const int slot = (int)(pt.launches % kPatchEvents);
        if (pt.on) {
            (void)hipEventRecord(pt.ev[slot][0], s);
            pt.cnt[slot] = count;
        }
        k_gd_cone_patch<<<pp, patch_threads(K, S), 0, s>>>(g, a, S);
        if (pt.on) {
            (void)hipEventRecord(pt.ev[slot][1], s);
            ++pt.launches;
        }
        if ((st = launch_status("k_gd_cone_patch"))) return st;
        if (cnt)
            k_gd_eval_part<<<grid_for(m, 1, kStreamGridCap), kBlock, 0, s>>>(g, t, owner, assigned, fv, gb[K % 3], 1,
                                                                              out + v * m, cnt, be);
        else
            k_gd_eval<<<grid_for(m, 1, kStreamGridCap), kBlock, 0, s>>>(g, t, owner, fv, gb[K % 3], 1, out + v * m, be);
        if ((st = launch_status("k_gd_eval"))) return st;
    }
    return 0;
}

}  // namespace

int akb_gd_cone_eval_f64(const double* x, const double* y, int nv, int nh, const uint8_t* diag, int npock,
                         const int32_t* ptri, const int32_t* pnbr, const int32_t* edge_tri, const int32_t* xptr,
                         const int32_t* xidx, const double* gx, int mx, const double* gy, int my, const double* f,
                         int nvals, int K, const double* omegas, void* work, int* owner, double* out,
                         unsigned long long* d_change, void* stream) {
    clear_error();
    AKB_REQUIRE(x && y && diag && gx && gy && f && omegas && work && owner && out && mx > 0 && my > 0 && nvals >= 1,
                "bad arguments");
    AKB_REQUIRE(K >= 1 && K <= kConeMaxK, "K sweeps in 1 .. 14");
    AKB_REQUIRE(nv >= 2 && nh >= 2, "grid of at least 2 x 2 points");
    for (int j = 2; j <= K; ++j) AKB_REQUIRE(omegas[j - 1] > 0 && omegas[j - 1] < 2, "Chebyshev weight outside (0, 2)");
    hipStream_t s = (hipStream_t)stream;
    Grid g{x, y, nv, nh, diag, npock, ptri, pnbr, edge_tri, xptr, xidx};
    Targets t{gx, gy, mx, my};
    int st = cone_claims(g, t, 1, owner, s, (uint8_t*)work + claim_scratch_offset(nv, nh, mx, my, nvals));
    if (st) return st;
    return cone_part(g, t, 0, (int64_t)nv * nh, 1, f, nvals, K, omegas, work, owner, out, nullptr, d_change, s);
}

// the single-process cone solve's begin: the target owners filled, then pass 1 with the cells' claims
// fused in (k_gd_cells_strip<true>); the axes (akb_gd_axes_f64) before it, the pockets' claims after
int akb_gd_cells_claims_f64(const double* x, const double* y, int nv, int nh, uint8_t* diag, double tol,
                            unsigned* d_flags, const double* gx, int mx, const double* gy, int my, int* owner,
                            void* stream) {
    clear_error();
    AKB_REQUIRE(x && y && diag && d_flags && gx && gy && owner && mx > 0 && my > 0, "bad arguments");
    AKB_REQUIRE(nv >= 2 && nh >= 2, "grid of at least 2 x 2 points");
    hipStream_t s = (hipStream_t)stream;
    const int64_t m = (int64_t)mx * my;
    k_fill_i32<<<grid_for(m, 4), kBlock, 0, s>>>(owner, m, INT32_MAX);
    int st = launch_status("k_fill_i32");
    if (st) return st;
    Grid g{x, y, nv, nh, diag, 0, nullptr, nullptr, nullptr, nullptr, nullptr};
    const TileClaims tc{Targets{gx, gy, mx, my}, owner};
    const StripGrid sg = strip_grid(nh, nv - 1);
    k_gd_cells_strip<true><<<sg.blocks, kStripThreads, 0, s>>>(g, diag, tol, d_flags, sg.seg_rows, tc);
    return launch_status("k_gd_cells_claims");
}

// the pockets' claims into owners the cells have claimed (akb_gd_cells_claims_f64)
int akb_gd_claim_pockets_f64(const double* x, const double* y, int nv, int nh, const uint8_t* diag, int npock,
                             const int32_t* ptri, const double* gx, int mx, const double* gy, int my, int* owner,
                             void* stream) {
    clear_error();
    AKB_REQUIRE(x && y && diag && gx && gy && owner && mx > 0 && my > 0 && nv >= 2 && nh >= 2, "bad arguments");
    if (npock == 0) return 0;
    AKB_REQUIRE(ptri, "pockets needed");
    Grid g{x, y, nv, nh, diag, npock, ptri, nullptr, nullptr, nullptr, nullptr};
    const int64_t pw = ((int64_t)npock + kBlock / 64 - 1) / (kBlock / 64);
    k_gd_claim_pockets<<<(unsigned)(pw < 16384 ? pw : 16384), kBlock, 0, (hipStream_t)stream>>>(g, Targets{gx, gy, mx, my},
                                                                                               owner);
    return launch_status("k_gd_claim_pockets");
}

// akb_gd_cone_eval_f64 on claimed owners: the solve and the evaluation only
int akb_gd_cone_solve_f64(const double* x, const double* y, int nv, int nh, const uint8_t* diag, int npock,
                          const int32_t* ptri, const int32_t* pnbr, const int32_t* edge_tri, const int32_t* xptr,
                          const int32_t* xidx, const double* gx, int mx, const double* gy, int my, const double* f,
                          int nvals, int K, const double* omegas, void* work, const int* owner, double* out,
                          unsigned long long* d_change, void* stream) {
    clear_error();
    AKB_REQUIRE(x && y && diag && gx && gy && f && omegas && work && owner && out && mx > 0 && my > 0 && nvals >= 1,
                "bad arguments");
    AKB_REQUIRE(K >= 1 && K <= kConeMaxK, "K sweeps in 1 .. 14");
    AKB_REQUIRE(nv >= 2 && nh >= 2, "grid of at least 2 x 2 points");
    AKB_REQUIRE(xptr && xidx && (npock == 0 || (ptri && pnbr && edge_tri)), "the band needs the pockets");
    for (int j = 2; j <= K; ++j) AKB_REQUIRE(omegas[j - 1] > 0 && omegas[j - 1] < 2, "Chebyshev weight outside (0, 2)");
    Grid g{x, y, nv, nh, diag, npock, ptri, pnbr, edge_tri, xptr, xidx};
    return cone_part(g, Targets{gx, gy, mx, my}, 0, (int64_t)nv * nh, 1, f, nvals, K, omegas, work, owner, out, nullptr,
                     d_change, (hipStream_t)stream);
}

int akb_gd_claims_f64(const double* x, const double* y, int nv, int nh, const uint8_t* diag, int npock,
                      const int32_t* ptri, const int32_t* pnbr, const int32_t* edge_tri, int row0, int row1,
                      int with_pockets, const double* gx, int mx, const double* gy, int my, int* owner, void* work,
                      void* stream) {
    clear_error();
    AKB_REQUIRE(x && y && diag && gx && gy && owner && mx > 0 && my > 0, "bad arguments");
    AKB_REQUIRE(nv >= 2 && nh >= 2 && row0 >= 0 && row1 <= nv - 1 && (row1 < 0 || row0 <= row1), "bad window");
    AKB_REQUIRE(!with_pockets || npock == 0 || (ptri && pnbr && edge_tri), "pockets needed");
    Grid g{x, y, nv, nh, diag, npock, ptri, pnbr, edge_tri, nullptr, nullptr};
    g.row0 = row0;
    g.row1 = row1;
    return cone_claims(g, Targets{gx, gy, mx, my}, with_pockets, owner, (hipStream_t)stream,
                       work ? (uint8_t*)work + claim_scratch_offset(nv, nh, mx, my, 1) : nullptr);
}

int akb_gd_cone_part_f64(const double* x, const double* y, int nv, int nh, const uint8_t* diag, int npock,
                         const int32_t* ptri, const int32_t* pnbr, const int32_t* edge_tri, const int32_t* xptr,
                         const int32_t* xidx, int64_t own0, int64_t own1, int band_on, const double* gx, int mx,
                         const double* gy, int my, const double* f, int nvals, int K, const double* omegas, void* work,
                         const int* owner, double* out, double* cnt, unsigned long long* d_change, void* stream) {
    clear_error();
    AKB_REQUIRE(x && y && diag && gx && gy && f && omegas && work && owner && out && cnt && mx > 0 && my > 0,
                "bad arguments");
    AKB_REQUIRE(nvals >= 1 && nvals <= 2, "one or two value sets");
    AKB_REQUIRE(K >= 1 && K <= kConeMaxK, "K sweeps in 1 .. 14");
    AKB_REQUIRE(!band_on || (xptr && xidx && (npock == 0 || (ptri && pnbr && edge_tri))), "the band needs the pockets");
    for (int j = 2; j <= K; ++j) AKB_REQUIRE(omegas[j - 1] > 0 && omegas[j - 1] < 2, "Chebyshev weight outside (0, 2)");
    Grid g{x, y, nv, nh, diag, npock, ptri, pnbr, edge_tri, xptr, xidx};
    return cone_part(g, Targets{gx, gy, mx, my}, own0, own1, band_on, f, nvals, K, omegas, work, owner, out, cnt,
                     d_change, (hipStream_t)stream);
}

int akb_gd_part_finish_f64(double* out, const double* cnt, int64_t m, int nvals, void* stream) {
    clear_error();
    AKB_REQUIRE(out && cnt && m > 0 && nvals >= 1, "bad arguments");
    k_gd_part_finish<<<grid_for(m), kBlock, 0, (hipStream_t)stream>>>(out, cnt, m, nvals);
    return launch_status("k_gd_part_finish");
}

int akb_gd_ring_f64(const double* x, const double* y, int nv, int nh, double* ring_x, double* ring_y, unsigned* d_flags,
                    void* stream) {
    clear_error();
    AKB_REQUIRE(x && y && ring_x && ring_y && d_flags && nv >= 2 && nh >= 2, "bad arguments");
    Grid g{x, y, nv, nh, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr};
    const int64_t L = 2 * (int64_t)(nh - 1) + 2 * (int64_t)(nv - 1);
    k_gd_ring<<<grid_for(L), kBlock, 0, (hipStream_t)stream>>>(g, ring_x, ring_y, d_flags);
    return launch_status("k_gd_ring");
}

int akb_gd_cells_window_f64(const double* x, const double* y, int nv, int nh, int row0, int row1, uint8_t* diag,
                            double tol, unsigned* d_flags, void* stream) {
    clear_error();
    AKB_REQUIRE(x && y && diag && d_flags && nv >= 2 && nh >= 2 && row0 >= 0 && row0 <= row1 && row1 <= nv - 1,
                "bad arguments");
    Grid g{x, y, nv, nh, diag, 0, nullptr, nullptr, nullptr, nullptr, nullptr};
    g.row0 = row0;
    g.row1 = row1;
    const int64_t wc = (int64_t)(row1 - row0) * (nh - 1);
    if (wc == 0) return 0;
    return launch_cells(g, diag, tol, d_flags, row1 - row0, (hipStream_t)stream);
}

// the patch timer's events and clock words (akb_release_all)
void akb_gd_release(void) {
    PatchTimer& t = patch_timer();
    if (!t.made) return;
    for (int k = 0; k < kPatchEvents; ++k)
        for (int q = 0; q < 2; ++q) {
            (void)hipEventDestroy(t.ev[k][q]);
            (void)hipEventDestroy(t.bev[k][q]);
        }
    (void)hipFree(t.clk);
    t.clk = nullptr;
    t.made = t.on = false;
    t.launches = t.band_launches = 0;
}

// diagnostics: k_gd_cone_patch launch times (see patch_timer)
int akb_gd_patch_timing(int enable) {
    clear_error();
    PatchTimer& t = patch_timer();
    if (enable && !t.made) {
        for (int k = 0; k < kPatchEvents; ++k)
            for (int q = 0; q < 2; ++q) {
                AKB_HIP_CHECK(hipEventCreate(&t.ev[k][q]));
                AKB_HIP_CHECK(hipEventCreate(&t.bev[k][q]));
            }
        AKB_HIP_CHECK(hipMalloc((void**)&t.clk, kPatchClk * sizeof(unsigned long long)));
        t.made = true;
    }
    if (enable) {  // a new record (stopping keeps the last one for akb_gd_patch_times / _phases)
        AKB_HIP_CHECK(hipMemset(t.clk, 0, kPatchClk * sizeof(unsigned long long)));
        t.launches = 0;
        t.band_launches = 0;
    }
    t.on = enable != 0;
    t.band_clk = enable == 2;
    return 0;
}

int akb_gd_patch_order(int K, uint16_t* out) {
    clear_error();
    AKB_REQUIRE(out && K >= 1 && K <= kConeMaxK, "K in 1 .. 14 and an output of 1024 entries");
    const int S = patch_split(K);
    AKB_REQUIRE(S >= 0, "no thread split for this K");
    patch_order_table(K, S, out);
    return S;
}

int akb_gd_patch_phases(unsigned long long* out) {
    clear_error();
    PatchTimer& t = patch_timer();
    AKB_REQUIRE(out, "null pointer");
    if (!t.made) {
        for (int k = 0; k < kPatchClk; ++k) out[k] = 0;
        return 0;
    }
    AKB_HIP_CHECK(hipDeviceSynchronize());
    AKB_HIP_CHECK(hipMemcpy(out, t.clk, kPatchClk * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return 0;
}

int akb_gd_patch_times(float* ms, int* cells, int max) {
    clear_error();
    PatchTimer& t = patch_timer();
    const int n = (int)std::min<int64_t>(std::min<int64_t>(t.launches, kPatchEvents), max);
    for (int k = 0; k < n; ++k) {
        const int slot = (int)((t.launches - n + k) % kPatchEvents);
        AKB_HIP_CHECK(hipEventSynchronize(t.ev[slot][1]));
        AKB_HIP_CHECK(hipEventElapsedTime(&ms[k], t.ev[slot][0], t.ev[slot][1]));
        if (cells) AKB_HIP_CHECK(hipMemcpy(&cells[k], t.cnt[slot], sizeof(int), hipMemcpyDeviceToHost));
    }
    return n;
}

int akb_gd_band_times(float* ms, int max) {
    clear_error();
    PatchTimer& t = patch_timer();
    const int n = (int)std::min<int64_t>(std::min<int64_t>(t.band_launches, kPatchEvents), max);
    for (int k = 0; k < n; ++k) {
        const int slot = (int)((t.band_launches - n + k) % kPatchEvents);
        AKB_HIP_CHECK(hipEventSynchronize(t.bev[slot][1]));
        AKB_HIP_CHECK(hipEventElapsedTime(&ms[k], t.bev[slot][0], t.bev[slot][1]));
    }
    return n;
}

}  // extern "C"

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
#include <type_traits>

#include "akb_common.h"
#include "akb_pairwise.h"

namespace akb {
namespace {

constexpr int kStripRowsDefault = 32;

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
    int no_xcd;  // 1: plain block order in the sweep (AKB_GD_NOXCD, A/B timing only)
    int strip_rows = kStripRowsDefault;  // rows per strip workgroup (AKB_GD_ROWS, A/B timing)
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
__global__ void __launch_bounds__(kBlock) k_gd_cells(Grid g, uint8_t* diag, double tol, unsigned* flags) {
    const int64_t nc = win_cell1(g);
    unsigned acc = 0;
    for (int64_t c = win_cell0(g) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < nc;
         c += (int64_t)gridDim.x * blockDim.x) {
        const int iv = (int)(c / (g.nh - 1)), ih = (int)(c - (int64_t)iv * (g.nh - 1));
        double bad = 0.0;
        const int d = cell_diag(g, iv, ih, &bad);
        diag[c] = (uint8_t)d;
        unsigned f = bad > 0 ? 1u : 0u;
        {   // bit 5: a non-finite point (a ray that missed); the ring kernel covers the last row / column
            const int64_t q = (int64_t)iv * g.nh + ih;
            if (!isfinite(g.x[q]) || !isfinite(g.y[q])) f |= 32u;
        }
        {   // every cell must share the grid's orientation (bits 3 / 4 both set: a folded grid)
            const int64_t q00 = (int64_t)iv * g.nh + ih;
            const double o = orient(g.x[q00], g.y[q00], g.x[q00 + 1], g.y[q00 + 1], g.x[q00 + g.nh + 1], g.y[q00 + g.nh + 1]);
            f |= o > 0 ? 8u : (o < 0 ? 16u : 1u);
        }
        const int64_t p00 = (int64_t)iv * g.nh + ih, p01 = p00 + 1, p10 = p00 + g.nh, p11 = p10 + 1;
        // right edge p01-p11 against the next cell's left triangle
        if (ih + 1 < g.nh - 1) {
            const int dn = cell_diag(g, iv, ih + 1, nullptr);
            const int64_t mine = d == 0 ? p00 : p10;           // opposite vertex of my right-edge triangle
            const int64_t other = dn == 0 ? p11 + 1 : p01 + 1;  // opposite vertex of its left-edge triangle
            const double x0 = g.x[p01], y0 = g.y[p01];
            const double ax = g.x[mine] - x0, ay = g.y[mine] - y0, cx = g.x[p11] - x0, cy = g.y[p11] - y0;
            const double ox = g.x[other] - x0, oy = g.y[other] - y0;
            const double s = fmax(fmax(fabs(ax), fabs(ay)), fmax(fmax(fabs(cx), fabs(cy)), fmax(fabs(ox), fabs(oy))));
            if (incircle(0.0, 0.0, ax, ay, cx, cy, ox, oy) > tol * s * s * s * s) f |= 2u;
        }
        // top edge p10-p11 against the next row's bottom triangle
        if (iv + 1 < g.nv - 1) {
            const int dn = cell_diag(g, iv + 1, ih, nullptr);
            const int64_t mine = d == 0 ? p00 : p01;
            const int64_t other = dn == 0 ? p11 + g.nh : p10 + g.nh;
            const double x0 = g.x[p10], y0 = g.y[p10];
            const double ax = g.x[mine] - x0, ay = g.y[mine] - y0, cx = g.x[p11] - x0, cy = g.y[p11] - y0;
            const double ox = g.x[other] - x0, oy = g.y[other] - y0;
            const double s = fmax(fmax(fabs(ax), fabs(ay)), fmax(fmax(fabs(cx), fabs(cy)), fmax(fabs(ox), fabs(oy))));
            if (incircle(0.0, 0.0, ax, ay, cx, cy, ox, oy) > tol * s * s * s * s) f |= 2u;
        }
        acc |= f;
    }
    // one atomic per wave, only for bits not yet set (every cell sets an orientation bit)
    for (int off = 32; off > 0; off >>= 1) acc |= __shfl_down(acc, off);
    if ((threadIdx.x & 63) == 0) {
        const unsigned cur = __hip_atomic_load(flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((cur | acc) != cur) atomicOr(flags, acc);
    }
}

// k_gd_cells on 16 x 16 tiles of the window's cells, one workgroup each: the tile's 18 x 18
// vertices in LDS (its cells, the next row's and column's), each of its 17 x 17 cells' diagonal
// formed once (cell_diag's arithmetic on the same values), then each cell's checks from LDS. Per
// cell: ~1.3 vertex loads and ~3 in-circle tests instead of ~10 and 5. Same diagonals and flags.
constexpr int kCellTile = 16;
__global__ void __launch_bounds__(kCellTile * kCellTile) k_gd_cells_tiled(Grid g, uint8_t* diag, double tol,
                                                                        unsigned* flags) {
    constexpr int T = kCellTile, V = T + 2;
    __shared__ double vx[V * V], vy[V * V];
    __shared__ uint8_t sdg[(T + 1) * (T + 1)];
    const int r_lo = g.row0, r_hi = g.row1 < 0 ? g.nv - 1 : g.row1;  // window cell rows [r_lo, r_hi)
    const int tiles_h = (g.nh - 1 + T - 1) / T;
    const int64_t ntiles = (int64_t)((r_hi - r_lo + T - 1) / T) * tiles_h;
    unsigned acc = 0;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int tv = (int)(tile / tiles_h), th = (int)(tile - (int64_t)tv * tiles_h);
        const int iv0 = r_lo + tv * T, ih0 = th * T;
        __syncthreads();
        for (int k = threadIdx.x; k < V * V; k += blockDim.x) {
            const int rr = k / V, cc = k - (k / V) * V;
            const int iv = iv0 + rr, ih = ih0 + cc;
            double x = 0.0, y = 0.0;
            if (iv < g.nv && ih < g.nh && iv <= r_hi + 1) {
                const int64_t q = (int64_t)iv * g.nh + ih;
                x = g.x[q];
                y = g.y[q];
            }
            vx[k] = x;
            vy[k] = y;
        }
        __syncthreads();
        // the diagonals of the tile's cells and of the next row / column (cell_diag's arithmetic)
        auto diag_of = [&](int rr, int cc, double* viol) {
            const int k00 = rr * V + cc, k01 = k00 + 1, k10 = k00 + V, k11 = k10 + 1;
            const double x0 = vx[k00], y0 = vy[k00];
            const double bx = vx[k01] - x0, by = vy[k01] - y0;
            const double cx = vx[k11] - x0, cy = vy[k11] - y0;
            const double dx = vx[k10] - x0, dy = vy[k10] - y0;
            const double ic = incircle(0.0, 0.0, bx, by, cx, cy, dx, dy);
            const int d = ic > 0 ? 1 : 0;
            if (viol) {
                const double sgn = d == 0 ? orient(0, 0, bx, by, cx, cy) * orient(0, 0, cx, cy, dx, dy)
                                          : orient(0, 0, bx, by, dx, dy) * orient(bx, by, cx, cy, dx, dy);
                *viol = sgn > 0 ? 0.0 : 1.0;
            }
            return d;
        };
        double bad = 0.0;
        const int rr = threadIdx.x / T, cc = threadIdx.x - (threadIdx.x / T) * T;
        const int iv = iv0 + rr, ih = ih0 + cc;
        const bool own = iv < r_hi && ih < g.nh - 1;
        const int d = own ? diag_of(rr, cc, &bad) : 0;
        sdg[rr * (T + 1) + cc] = (uint8_t)d;
        if (threadIdx.x < 2 * T + 1) {  // the next row (T + 1 cells) and column (T cells)
            const int r2 = threadIdx.x <= T ? T : (int)threadIdx.x - (T + 1);
            const int c2 = threadIdx.x <= T ? (int)threadIdx.x : T;
            const int jv = iv0 + r2, jh = ih0 + c2;
            sdg[r2 * (T + 1) + c2] =
                (jv < g.nv - 1 && jh < g.nh - 1 && jv <= r_hi) ? (uint8_t)diag_of(r2, c2, nullptr) : (uint8_t)0;
        }
        __syncthreads();
        if (!own) continue;
        const int64_t c = (int64_t)iv * (g.nh - 1) + ih;
        diag[c] = (uint8_t)d;
        unsigned f = bad > 0 ? 1u : 0u;
        const int k00 = rr * V + cc, k01 = k00 + 1, k10 = k00 + V, k11 = k10 + 1;
        if (!isfinite(vx[k00]) || !isfinite(vy[k00])) f |= 32u;
        {
            const double o = orient(vx[k00], vy[k00], vx[k01], vy[k01], vx[k11], vy[k11]);
            f |= o > 0 ? 8u : (o < 0 ? 16u : 1u);
        }
        if (ih + 1 < g.nh - 1) {  // right edge p01-p11 against the next cell's left triangle
            const int dn = sdg[rr * (T + 1) + cc + 1];
            const int mine = d == 0 ? k00 : k10, other = dn == 0 ? k11 + 1 : k01 + 1;
            const double x0 = vx[k01], y0 = vy[k01];
            const double ax = vx[mine] - x0, ay = vy[mine] - y0, cx = vx[k11] - x0, cy = vy[k11] - y0;
            const double ox = vx[other] - x0, oy = vy[other] - y0;
            const double sc = fmax(fmax(fabs(ax), fabs(ay)), fmax(fmax(fabs(cx), fabs(cy)), fmax(fabs(ox), fabs(oy))));
            if (incircle(0.0, 0.0, ax, ay, cx, cy, ox, oy) > tol * sc * sc * sc * sc) f |= 2u;
        }
        if (iv + 1 < g.nv - 1) {  // top edge p10-p11 against the next row's bottom triangle
            const int dn = sdg[(rr + 1) * (T + 1) + cc];
            const int mine = d == 0 ? k00 : k01, other = dn == 0 ? k11 + V : k10 + V;
            const double x0 = vx[k10], y0 = vy[k10];
            const double ax = vx[mine] - x0, ay = vy[mine] - y0, cx = vx[k11] - x0, cy = vy[k11] - y0;
            const double ox = vx[other] - x0, oy = vy[other] - y0;
            const double sc = fmax(fmax(fabs(ax), fabs(ay)), fmax(fmax(fabs(cx), fabs(cy)), fmax(fabs(ox), fabs(oy))));
            if (incircle(0.0, 0.0, ax, ay, cx, cy, ox, oy) > tol * sc * sc * sc * sc) f |= 2u;
        }
        acc |= f;
    }
    for (int off = 32; off > 0; off >>= 1) acc |= __shfl_down(acc, off);
    if ((threadIdx.x & 63) == 0) {
        const unsigned cur = __hip_atomic_load(flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((cur | acc) != cur) atomicOr(flags, acc);
    }
}

// ring positions -> coordinates, for the host pocket builder (bit 5 of flags: a non-finite one)
__global__ void k_gd_ring(Grid g, double* rx, double* ry, unsigned* flags) {
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

__device__ __forceinline__ int64_t ring_pos(const Grid& g, int iv, int ih) {
    const int64_t a = g.nh - 1, b = g.nv - 1;
    if (iv == 0) return ih;
    if (ih == g.nh - 1) return a + iv;
    if (iv == g.nv - 1) return a + b + (g.nh - 1 - ih);
    if (ih == 0) return 2 * a + b + (g.nv - 1 - iv);
    return -1;
}

// sums of the local problem: Q (geometry only, shared by the value sets; the factor 4 applied at
// the solve) and s per value set
template <int NV>
struct GradAcc {
    double q0 = 0, q1 = 0, q3 = 0;
    double s0[NV] = {}, s1[NV] = {};
};

constexpr int64_t kGradChunk = 4 * kBlock;  // vertices per workgroup of a sweep

// one edge (vertex i -> j) of the local problem, NV value sets
template <int NV>
__device__ __forceinline__ void grad_edge(const Grid& g, int64_t n, int64_t j, double xi, double yi,
                                          const double (&fi)[NV], const double* __restrict__ f,
                                          const double* __restrict__ gin, GradAcc<NV>& A) {
    const double ex = g.x[j] - xi, ey = g.y[j] - yi;
    // 1 / L^3 from the hardware reciprocal square root and one Newton step (relative error
    // ~1e-16: this solve is converged to 1e-10, not reproduced bit for bit)
    const double l2 = ex * ex + ey * ey;
    double r = __builtin_amdgcn_rsq(l2);
    r = r * __builtin_fma(-0.5 * l2 * r, r, 1.5);
    const double r3 = r * r * r;
    const double wx = ex * r3, wy = ey * r3;
    A.q0 = __builtin_fma(ex, wx, A.q0);
    A.q1 = __builtin_fma(ex, wy, A.q1);
    A.q3 = __builtin_fma(ey, wy, A.q3);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const double df2 = -ex * gin[2 * (v * n + j)] - ey * gin[2 * (v * n + j) + 1];
        const double w = 6 * (fi[v] - f[v * n + j]) - 2 * df2;
        A.s0[v] = __builtin_fma(w, wx, A.s0[v]);
        A.s1[v] = __builtin_fma(w, wy, A.s1[v]);
    }
}

// Chebyshev semi-iteration on top of the Jacobi sweep (gprev != nullptr): the new gradient is
// omega * (y - g_prev) + g_prev with y the Jacobi solve's value, which contracts the error by
// ~0.27 per sweep instead of Jacobi's ~1/2 (the iteration matrix's spectrum lies in [-1/2, 1/2]:
// the local problem is block diagonally dominant by a factor 2)
struct Cheb {
    const double* gprev;  // the iterate before gin (nullptr: a plain sweep, unless zero_prev)
    double omega;
    int zero_prev = 0;    // the previous iterate is zero (a Chebyshev step from x_0 = 0)
};

// the 2 x 2 solve of value set v; returns the relative change of the Jacobi step (scipy's measure)
template <int NV>
__device__ __forceinline__ double grad_solve(const GradAcc<NV>& A, int v, const double* gin, double* gout,
                                             int64_t o, const Cheb& ch) {
    const double q0 = 4 * A.q0, q1 = 4 * A.q1, q3 = 4 * A.q3;
    const double inv = 1.0 / (q0 * q3 - q1 * q1);
    const double r0 = (q3 * A.s0[v] - q1 * A.s1[v]) * inv;
    const double r1 = (-q1 * A.s0[v] + q0 * A.s1[v]) * inv;
    const double c = fmax(fabs(gin[o] + r0), fabs(gin[o + 1] + r1)) / fmax(1.0, fmax(fabs(r0), fabs(r1)));
    if (ch.gprev) {
        const double p0 = ch.gprev[o], p1 = ch.gprev[o + 1];
        gout[o] = ch.omega * (-r0 - p0) + p0;
        gout[o + 1] = ch.omega * (-r1 - p1) + p1;
    } else if (ch.zero_prev) {
        gout[o] = ch.omega * (-r0 - 0.0) + 0.0;
        gout[o + 1] = ch.omega * (-r1 - 0.0) + 0.0;
    } else {
        gout[o] = -r0;
        gout[o + 1] = -r1;
    }
    return c;
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

__device__ __forceinline__ void change_max(double worst, unsigned long long* chg) {
    __shared__ double red[kBlock / 64];
    for (int off = 32; off > 0; off >>= 1) worst = fmax(worst, __shfl_down(worst, off));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = worst;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / 64; ++w) worst = fmax(worst, red[w]);
        const unsigned long long bits = (unsigned long long)__double_as_longlong(worst);
        if (chg && worst > 0 && __hip_atomic_load(chg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < bits)
            atomicMax(chg, bits);
    }
}

// One Jacobi sweep for NV value sets sharing the geometry: gout[i] from gin of the grid
// neighbours (4 axis + the diagonals of the 4 cells around i). Ring vertices also have pocket
// chords - a hull vertex can fan out to thousands - so for them this kernel only stores the
// grid-edge sums in ring_acc and k_gd_grad_ring adds the chords with a whole wave and solves.
template <int NV>
__global__ void __launch_bounds__(kBlock) k_gd_grad(Grid g, const double* __restrict__ f,
                                                    const double* __restrict__ gin, double* __restrict__ gout,
                                                    double* __restrict__ ring_acc, unsigned long long* chg, Cheb ch) {
    const int64_t n = (int64_t)g.nv * g.nh;
    double worst = 0.0;
    // XCD-aware: the grid is a multiple of 8 and blocks b, b + 8, ... (one XCD, dealt round-robin)
    // take consecutive chunks, so the rows above and below a chunk are read through the same L2
    const int64_t per = gridDim.x / 8;
    const int64_t chunk = g.no_xcd ? (int64_t)blockIdx.x : (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
    const int64_t i0 = chunk * kGradChunk, i1 = i0 + kGradChunk < n ? i0 + kGradChunk : n;
    for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
        const int iv = (int)(i / g.nh), ih = (int)(i - (int64_t)iv * g.nh);
        const double xi = g.x[i], yi = g.y[i];
        double fi[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) fi[v] = f[v * n + i];
        GradAcc<NV> A;
        if (ih > 0) grad_edge<NV>(g, n, i - 1, xi, yi, fi, f, gin, A);
        if (ih < g.nh - 1) grad_edge<NV>(g, n, i + 1, xi, yi, fi, f, gin, A);
        if (iv > 0) grad_edge<NV>(g, n, i - g.nh, xi, yi, fi, f, gin, A);
        if (iv < g.nv - 1) grad_edge<NV>(g, n, i + g.nh, xi, yi, fi, f, gin, A);
        const int64_t c0 = (int64_t)iv * (g.nh - 1) + ih;  // cell with p00 = i
        if (iv > 0 && ih > 0 && g.diag[c0 - g.nh] == 0) grad_edge<NV>(g, n, i - g.nh - 1, xi, yi, fi, f, gin, A);
        if (iv > 0 && ih < g.nh - 1 && g.diag[c0 - (g.nh - 1)] == 1)
            grad_edge<NV>(g, n, i - g.nh + 1, xi, yi, fi, f, gin, A);
        if (iv < g.nv - 1 && ih > 0 && g.diag[c0 - 1] == 1) grad_edge<NV>(g, n, i + g.nh - 1, xi, yi, fi, f, gin, A);
        if (iv < g.nv - 1 && ih < g.nh - 1 && g.diag[c0] == 0) grad_edge<NV>(g, n, i + g.nh + 1, xi, yi, fi, f, gin, A);
        const int64_t r = ring_pos(g, iv, ih);
        if (r >= 0) {
            double* d = ring_acc + r * (3 + 2 * NV);
            d[0] = A.q0;
            d[1] = A.q1;
            d[2] = A.q3;
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                d[3 + 2 * v] = A.s0[v];
                d[4 + 2 * v] = A.s1[v];
            }
            continue;
        }
#pragma unroll
        for (int v = 0; v < NV; ++v) worst = fmax(worst, grad_solve<NV>(A, v, gin, gout, 2 * (v * n + i), ch));
    }
    change_max(worst, chg);
}

// The same sweep with every vertex's data read from HBM once: a workgroup walks down a strip of
// kStripW columns (plus one halo column each side) over strip_rows rows (default 32), holding three rows of
// (x, y, f, g) in an LDS ring, the next row already in registers while the current one is solved
// (its loads in flight across the row's arithmetic). The per-vertex edge order and arithmetic are
// k_gd_grad's, so both give the same bits; the global version's eight-neighbour gathers (about 50
// load instructions per vertex through the texture path) become LDS reads.

template <int NV, int W>
struct StripRow {  // one row of a strip in LDS: column c of the strip at [c + 1], halos at 0 / W + 1
    double x[W + 2], y[W + 2];
    double f[NV][W + 2];
    double gx[NV][W + 2], gy[NV][W + 2];
    uint8_t d[W + 2];  // the diagonal flags of the cell row below (cells (row, col - 1) at [col])
};

template <int NV>
struct StripVals {
    double x, y, f[NV], gx[NV], gy[NV];
    int d;  // diag of cell (row, col) (0 outside the cells)
};

template <int NV>
__device__ __forceinline__ void strip_load(const Grid& g, int64_t n, const double* __restrict__ f,
                                           const double* __restrict__ gin, int64_t i, StripVals<NV>& v) {
    v.x = g.x[i];
    v.y = g.y[i];
    const int iv = (int)(i / g.nh), ih = (int)(i - (int64_t)iv * g.nh);
    v.d = (iv < g.nv - 1 && ih < g.nh - 1) ? g.diag[(int64_t)iv * (g.nh - 1) + ih] : 0;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        v.f[k] = f[k * n + i];
        v.gx[k] = gin[2 * (k * n + i)];
        v.gy[k] = gin[2 * (k * n + i) + 1];
    }
}

template <int NV, int W>
__device__ __forceinline__ void strip_store(StripRow<NV, W>& r, int c, const StripVals<NV>& v) {
    r.x[c] = v.x;
    r.y[c] = v.y;
    r.d[c] = (uint8_t)v.d;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        r.f[k][c] = v.f[k];
        r.gx[k][c] = v.gx[k];
        r.gy[k][c] = v.gy[k];
    }
}

// grad_edge with the neighbour's data from an LDS row
template <int NV, int W>
__device__ __forceinline__ void grad_edge_lds(const StripRow<NV, W>& r, int c, double xi, double yi,
                                              const double (&fi)[NV], GradAcc<NV>& A) {
    const double ex = r.x[c] - xi, ey = r.y[c] - yi;
    const double l2 = ex * ex + ey * ey;
    double rr = __builtin_amdgcn_rsq(l2);
    rr = rr * __builtin_fma(-0.5 * l2 * rr, rr, 1.5);
    const double r3 = rr * rr * rr;
    const double wx = ex * r3, wy = ey * r3;
    A.q0 = __builtin_fma(ex, wx, A.q0);
    A.q1 = __builtin_fma(ex, wy, A.q1);
    A.q3 = __builtin_fma(ey, wy, A.q3);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const double df2 = -ex * r.gx[v][c] - ey * r.gy[v][c];
        const double w = 6 * (fi[v] - r.f[v][c]) - 2 * df2;
        A.s0[v] = __builtin_fma(w, wx, A.s0[v]);
        A.s1[v] = __builtin_fma(w, wy, A.s1[v]);
    }
}

// kGS: a line Gauss-Seidel sweep instead of Jacobi - once row iv is solved, its new gradients
// replace the old ones in the LDS ring, so row iv + 1 sees its upper neighbours' new values (the
// way scipy's Gauss-Seidel sweep sees its earlier vertices'); left / right neighbours, the rows
// outside the chunk, the halo columns and the ring vertices keep the old values. Same local solve,
// same fixed point, ~1/3 fewer sweeps; deterministic (no value depends on workgroup timing).
template <int NV, int W, bool kGS = false>
__global__ void __launch_bounds__(W) k_gd_grad_strip(Grid g, const double* __restrict__ f,
                                                     const double* __restrict__ gin, double* __restrict__ gout,
                                                     double* __restrict__ ring_acc, unsigned long long* chg, Cheb ch) {
    constexpr int kStripW = W;
    __shared__ StripRow<NV, W> R[3];
    const int64_t n = (int64_t)g.nv * g.nh;
    const int nstrips = (g.nh + kStripW - 1) / kStripW;
    const int strip = blockIdx.x % nstrips, chunk = blockIdx.x / nstrips;
    const int c0 = strip * kStripW;
    const int r0 = chunk * g.strip_rows;
    const int r1 = r0 + g.strip_rows < g.nv ? r0 + g.strip_rows : g.nv;
    const int t = threadIdx.x;
    const int ih = c0 + t;
    const bool col = ih < g.nh;
    // halo columns: thread 0 the left one, thread 1 the right one (when they exist)
    const int hcol = t == 0 ? c0 - 1 : c0 + kStripW;
    const int hslot = t == 0 ? 0 : kStripW + 1;
    const bool halo = t < 2 && hcol >= 0 && hcol < g.nh;
    double worst = 0.0;
    // rows iv + 1 and iv + 2 wait in two register sets (a and b, alternating) while row iv is solved
    StripVals<NV> a, ah, b, bh;
    auto load_row = [&](int rr, StripVals<NV>& v, StripVals<NV>& vh) {
        if (col) strip_load<NV>(g, n, f, gin, (int64_t)rr * g.nh + ih, v);
        if (halo) strip_load<NV>(g, n, f, gin, (int64_t)rr * g.nh + hcol, vh);
    };
    auto store_row = [&](int rr, const StripVals<NV>& v, const StripVals<NV>& vh) {
        if (col) strip_store<NV, W>(R[rr % 3], t + 1, v);
        if (halo) strip_store<NV, W>(R[rr % 3], hslot, vh);
    };
    // prologue: rows r0 - 1 and r0 into LDS, rows r0 + 1 and r0 + 2 into registers (a row k is
    // needed while k <= r1: row r1 is the last row's lower neighbour)
    for (int rr = r0 - 1; rr <= r0; ++rr) {
        if (rr < 0) continue;
        load_row(rr, a, ah);
        store_row(rr, a, ah);
    }
    if (r0 + 1 < g.nv) load_row(r0 + 1, a, ah);
    if (r0 + 2 < g.nv && r0 + 2 <= r1) load_row(r0 + 2, b, bh);
    double ngx[NV], ngy[NV];
    bool solved = false;
    auto step = [&](int iv, StripVals<NV>& nx, StripVals<NV>& nh_) {
        if (iv + 1 < g.nv) store_row(iv + 1, nx, nh_);  // row iv + 1: registers -> LDS
        __syncthreads();
        if (iv + 3 < g.nv && iv + 3 <= r1) load_row(iv + 3, nx, nh_);  // two rows ahead
        if (col) {
            const StripRow<NV, W>& up = R[(iv + 2) % 3];  // row iv - 1
            const StripRow<NV, W>& cur = R[iv % 3];
            const StripRow<NV, W>& dn = R[(iv + 1) % 3];
            const int c = t + 1;
            const int64_t i = (int64_t)iv * g.nh + ih;
            const double xi = cur.x[c], yi = cur.y[c];
            double fi[NV];
#pragma unroll
            for (int v = 0; v < NV; ++v) fi[v] = cur.f[v][c];
            GradAcc<NV> A;
            if (ih > 0) grad_edge_lds<NV, W>(cur, c - 1, xi, yi, fi, A);
            if (ih < g.nh - 1) grad_edge_lds<NV, W>(cur, c + 1, xi, yi, fi, A);
            if (iv > 0) grad_edge_lds<NV, W>(up, c, xi, yi, fi, A);
            if (iv < g.nv - 1) grad_edge_lds<NV, W>(dn, c, xi, yi, fi, A);
            // the four cells around i: (iv - 1, ih - 1), (iv - 1, ih), (iv, ih - 1), (iv, ih)
            if (iv > 0 && ih > 0 && up.d[c - 1] == 0) grad_edge_lds<NV, W>(up, c - 1, xi, yi, fi, A);
            if (iv > 0 && ih < g.nh - 1 && up.d[c] == 1) grad_edge_lds<NV, W>(up, c + 1, xi, yi, fi, A);
            if (iv < g.nv - 1 && ih > 0 && cur.d[c - 1] == 1) grad_edge_lds<NV, W>(dn, c - 1, xi, yi, fi, A);
            if (iv < g.nv - 1 && ih < g.nh - 1 && cur.d[c] == 0) grad_edge_lds<NV, W>(dn, c + 1, xi, yi, fi, A);
            const int64_t r = ring_pos(g, iv, ih);
            if (r >= 0) {
                double* d = ring_acc + r * (3 + 2 * NV);
                d[0] = A.q0;
                d[1] = A.q1;
                d[2] = A.q3;
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    d[3 + 2 * v] = A.s0[v];
                    d[4 + 2 * v] = A.s1[v];
                }
            } else {
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    const int64_t o = 2 * (v * n + i);
                    worst = fmax(worst, grad_solve<NV>(A, v, gin, gout, o, ch));
                    if (kGS) {
                        ngx[v] = gout[o];
                        ngy[v] = gout[o + 1];
                    }
                }
                solved = kGS;
            }
        }
        __syncthreads();  // the next step overwrites row iv - 1's slot
        if (kGS && solved) {  // row iv's new gradients, for row iv + 1 (read after the next sync)
            StripRow<NV, W>& cur = R[iv % 3];
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                cur.gx[v][t + 1] = ngx[v];
                cur.gy[v][t + 1] = ngy[v];
            }
            solved = false;
        }
    };
    for (int iv = r0; iv < r1; iv += 2) {
        step(iv, a, ah);
        if (iv + 1 < r1) step(iv + 1, b, bh);
    }
    change_max_n<W>(worst, chg);
}

// ring vertices: one wave each adds the pocket chords (lanes stride the chord list, fixed-order
// wave reduction) to the grid-edge sums, then solves
template <int NV>
__global__ void __launch_bounds__(kBlock) k_gd_grad_ring(Grid g, const double* __restrict__ f,
                                                         const double* __restrict__ gin, double* __restrict__ gout,
                                                         const double* __restrict__ ring_acc, unsigned long long* chg,
                                                         Cheb ch) {
    const int64_t n = (int64_t)g.nv * g.nh;
    const int64_t a = g.nh - 1, b = g.nv - 1, L = 2 * a + 2 * b;
    const int lane = threadIdx.x & 63;
    double worst = 0.0;
    for (int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; r < L;
         r += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        int64_t i;
        if (r < a) i = r;
        else if (r < a + b) i = (r - a) * g.nh + (g.nh - 1);
        else if (r < 2 * a + b) i = (int64_t)(g.nv - 1) * g.nh + (g.nh - 1 - (r - a - b));
        else i = (int64_t)(g.nv - 1 - (r - 2 * a - b)) * g.nh;
        const double xi = g.x[i], yi = g.y[i];
        double fi[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) fi[v] = f[v * n + i];
        GradAcc<NV> A;
        for (int32_t k = g.xptr[r] + lane; k < g.xptr[r + 1]; k += 64) grad_edge<NV>(g, n, g.xidx[k], xi, yi, fi, f, gin, A);
        for (int off = 32; off > 0; off >>= 1) {
            A.q0 += __shfl_down(A.q0, off);
            A.q1 += __shfl_down(A.q1, off);
            A.q3 += __shfl_down(A.q3, off);
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                A.s0[v] += __shfl_down(A.s0[v], off);
                A.s1[v] += __shfl_down(A.s1[v], off);
            }
        }
        if (lane == 0) {
            const double* d = ring_acc + r * (3 + 2 * NV);
            A.q0 += d[0];
            A.q1 += d[1];
            A.q3 += d[2];
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                A.s0[v] += d[3 + 2 * v];
                A.s1[v] += d[4 + 2 * v];
            }
#pragma unroll
            for (int v = 0; v < NV; ++v) worst = fmax(worst, grad_solve<NV>(A, v, gin, gout, 2 * (v * n + i), ch));
        }
    }
    change_max(worst, chg);
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
// sums and k_gd_grad_ring adds the chords of x_{k+1} and solves after the launch. Per vertex the
// edge order and arithmetic are k_gd_grad's, so kK sweeps here give the bits of kK sweeps there.

// lane l gets lane l - 1's value (DPP wave_shr:1; lane 0 keeps its own) / lane l + 1's (wave_shl:1)
__device__ __forceinline__ int lane_prev_i(int v) { return __builtin_amdgcn_update_dpp(v, v, 0x138, 0xf, 0xf, false); }
__device__ __forceinline__ int lane_next_i(int v) { return __builtin_amdgcn_update_dpp(v, v, 0x130, 0xf, 0xf, false); }
// (the cell flags are loaded per lane rather than shifted: an int shifted this way read the
// neighbour on the wrong side at a flag change on the MI355X, tests/test_gpu_parity.py's 300 x 280
// lattice; the doubles' shifts are checked bit for bit against the LDS kernels there)
// doubles: one v_mov_b32_dpp per half with bound_ctrl (lane 0 / lane 63 read 0: halo lanes)
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

// grad_edge with the neighbour in registers
template <int NV>
__device__ __forceinline__ void edge_rv(const RV<NV>& o, double xi, double yi, const double (&fi)[NV],
                                        GradAcc<NV>& A) {
    const double ex = o.x - xi, ey = o.y - yi;
    const double l2 = ex * ex + ey * ey;
    double rr = __builtin_amdgcn_rsq(l2);
    rr = rr * __builtin_fma(-0.5 * l2 * rr, rr, 1.5);
    const double r3 = rr * rr * rr;
    const double wx = ex * r3, wy = ey * r3;
    A.q0 = __builtin_fma(ex, wx, A.q0);
    A.q1 = __builtin_fma(ex, wy, A.q1);
    A.q3 = __builtin_fma(ey, wy, A.q3);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const double df2 = -ex * o.gx[v] - ey * o.gy[v];
        const double w = 6 * (fi[v] - o.f[v]) - 2 * df2;
        A.s0[v] = __builtin_fma(w, wx, A.s0[v]);
        A.s1[v] = __builtin_fma(w, wy, A.s1[v]);
    }
}

// the grid-edge sums of the vertex in row `cur` (wave-uniform control flow: the lane shifts run in
// every lane; only the shifts some lane of the wave needs are made)
template <int NV>
__device__ __forceinline__ GradAcc<NV> vertex_sums(const RV<NV>& up, const RV<NV>& cur, const RV<NV>& dn,
                                                   bool hl, bool hr, bool hu, bool hd) {
    // which diagonals exist: cells (iv - 1, ih - 1), (iv - 1, ih), (iv, ih - 1), (iv, ih)
    const bool ul = hu && hl && up.dl == 0, ur = hu && hr && up.d == 1;
    const bool dl = hd && hl && cur.dl == 1, dr = hd && hr && cur.d == 0;
    GradAcc<NV> A;
    // one shifted neighbour live at a time, the edges in k_gd_grad's order
    {
        const RV<NV> L = rv_shift<NV, false>(cur);
        if (hl) edge_rv<NV>(L, cur.x, cur.y, cur.f, A);
    }
    {
        const RV<NV> R = rv_shift<NV, true>(cur);
        if (hr) edge_rv<NV>(R, cur.x, cur.y, cur.f, A);
    }
    if (hu) edge_rv<NV>(up, cur.x, cur.y, cur.f, A);
    if (hd) edge_rv<NV>(dn, cur.x, cur.y, cur.f, A);
    if (__any(ul)) {
        const RV<NV> N = rv_shift<NV, false>(up);
        if (ul) edge_rv<NV>(N, cur.x, cur.y, cur.f, A);
    }
    if (__any(ur)) {
        const RV<NV> N = rv_shift<NV, true>(up);
        if (ur) edge_rv<NV>(N, cur.x, cur.y, cur.f, A);
    }
    if (__any(dl)) {
        const RV<NV> N = rv_shift<NV, false>(dn);
        if (dl) edge_rv<NV>(N, cur.x, cur.y, cur.f, A);
    }
    if (__any(dr)) {
        const RV<NV> N = rv_shift<NV, true>(dn);
        if (dr) edge_rv<NV>(N, cur.x, cur.y, cur.f, A);
    }
    return A;
}

// grad_solve on registers: y = -Q^-1 s, the change against the current value (gi), then the
// Chebyshev combination with the previous iterate (p; plain: y itself)
template <int NV>
__device__ __forceinline__ double solve_rv(const GradAcc<NV>& A, int v, double gix, double giy, bool plain,
                                           double omega, double px, double py, double& ox, double& oy) {
    const double q0 = 4 * A.q0, q1 = 4 * A.q1, q3 = 4 * A.q3;
    const double inv = 1.0 / (q0 * q3 - q1 * q1);  // the same for every v: CSE'd across the unrolled calls
    const double r0 = (q3 * A.s0[v] - q1 * A.s1[v]) * inv;
    const double r1 = (-q1 * A.s0[v] + q0 * A.s1[v]) * inv;
    const double c = fmax(fabs(gix + r0), fabs(giy + r1)) / fmax(1.0, fmax(fabs(r0), fabs(r1)));
    if (plain) {
        ox = -r0;
        oy = -r1;
    } else {
        ox = omega * (-r0 - px) + px;
        oy = omega * (-r1 - py) + py;
    }
    return c;
}

template <int NV>
struct SweepArgs {
    const double* f;       // (NV, n) values
    const double* gin;     // (NV, n, 2) x_k, nullptr = zeros
    const double* gprev;   // (NV, n, 2) x_{k-1} for the first sweep's Chebyshev step, nullptr = plain
    double om1, om2;       // the two sweeps' weights
    double* gout1;         // x_{k+1}
    double* gout2;         // x_{k+2} (kK = 2)
    const double* chords;  // (L, 3 + 2 NV) pocket-chord sums of x_k (k_gd_ring_chords)
    double* ring_acc;      // (L, 3 + 2 NV) grid-edge sums of x_{k+1} at ring vertices (kK = 2)
    unsigned long long* chg;  // [2]: largest relative change of each sweep
    int rows;              // rows per wave
};

template <int NV, int kK, int kWaves, int kDepth = 1>
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
        // sweep 1 of row i (rows up / cur / dn) -> s (x_{k+1} of row i, NV x 2)
        auto sweep1 = [&](int i, const RV<NV>& up, const RV<NV>& cur, const RV<NV>& dn, const double (&px)[NV],
                          const double (&py)[NV], RV<NV>& s) {
            s = cur;  // geometry and values carry over; gradients replaced below
            GradAcc<NV> A = vertex_sums<NV>(up, cur, dn, hl, hr, i > 0, i < g.nv - 1);
            if (!col || i < 0 || i >= g.nv) return;
            const int64_t r = ring_pos(g, i, ih);
            if (r >= 0) {  // pocket chords of x_k (commutative sum: the bits of k_gd_grad_ring's order)
                const double* c = a.chords + r * (3 + 2 * NV);
                A.q0 = c[0] + A.q0;
                A.q1 = c[1] + A.q1;
                A.q3 = c[2] + A.q3;
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    A.s0[v] = c[3 + 2 * v] + A.s0[v];
                    A.s1[v] = c[4 + 2 * v] + A.s1[v];
                }
            }
            const bool mine = own && i >= r0 && i < r1;
            const int64_t o = (int64_t)i * g.nh + ih;
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                double ox, oy;
                const double ch = solve_rv<NV>(A, v, cur.gx[v], cur.gy[v], a.gprev == nullptr, a.om1, px[v], py[v],
                                               ox, oy);
                s.gx[v] = ox;
                s.gy[v] = oy;
                if (mine) {
                    worst1 = fmax(worst1, ch);
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
        // rows i + 2 (and, kDepth = 2, i + 3) in flight across row i's arithmetic: the VGPR budget
        // of two waves per SIMD holds a second prefetched row
        RV<NV> P;
        double sx[NV], sy[NV];
        if (kDepth == 2) {
            load(first + 2, P);
            load_prev(first + 1, sx, sy);
        }
        for (int i = first; i <= last; ++i) {
            RV<NV> N;
            if (kDepth == 2) {
                N = P;
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    qx[v] = sx[v];
                    qy[v] = sy[v];
                }
                load(i + 3, P);
                load_prev(i + 2, sx, sy);
            } else {
                load(i + 2, N);
                load_prev(i + 1, qx, qy);
            }
            sweep1(i, G1, G2, G3, px, py, S2);
            if (kK == 2 && i - 1 >= r0 && i - 1 < r1) {
                // sweep 2 of row i - 1 from the x_{k+1} rows S0 (i - 2), S1 (i - 1), S2 (i)
                const int iv = i - 1;
                GradAcc<NV> A = vertex_sums<NV>(S0, S1, S2, hl, hr, iv > 0, iv < g.nv - 1);
                if (own) {
                    const int64_t o = (int64_t)iv * g.nh + ih;
                    const int64_t r = ring_pos(g, iv, ih);
                    if (r >= 0) {  // k_gd_grad_ring adds the chords of x_{k+1} and solves
                        double* d = a.ring_acc + r * (3 + 2 * NV);
                        d[0] = A.q0;
                        d[1] = A.q1;
                        d[2] = A.q3;
#pragma unroll
                        for (int v = 0; v < NV; ++v) {
                            d[3 + 2 * v] = A.s0[v];
                            d[4 + 2 * v] = A.s1[v];
                        }
                    } else {
#pragma unroll
                        for (int v = 0; v < NV; ++v) {
                            double ox, oy;
                            // Chebyshev against x_k of row i - 1 (G1)
                            worst2 = fmax(worst2, solve_rv<NV>(A, v, S1.gx[v], S1.gy[v], false, a.om2, G1.gx[v],
                                                               G1.gy[v], ox, oy));
                            a.gout2[2 * (v * n + o)] = ox;
                            a.gout2[2 * (v * n + o) + 1] = oy;
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

// pocket-chord sums of every ring vertex from gradients gin (nullptr = zeros): one wave per ring
// vertex, lanes striding its chord list, the fixed-order wave reduction of k_gd_grad_ring
template <int NV>
__global__ void __launch_bounds__(kBlock) k_gd_ring_chords(Grid g, const double* __restrict__ f,
                                                           const double* __restrict__ gin, double* __restrict__ out) {
    const int64_t n = (int64_t)g.nv * g.nh;
    const int64_t a = g.nh - 1, b = g.nv - 1, L = 2 * a + 2 * b;
    const int lane = threadIdx.x & 63;
    for (int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; r < L;
         r += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        int64_t i;
        if (r < a) i = r;
        else if (r < a + b) i = (r - a) * g.nh + (g.nh - 1);
        else if (r < 2 * a + b) i = (int64_t)(g.nv - 1) * g.nh + (g.nh - 1 - (r - a - b));
        else i = (int64_t)(g.nv - 1 - (r - 2 * a - b)) * g.nh;
        const double xi = g.x[i], yi = g.y[i];
        double fi[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) fi[v] = f[v * n + i];
        GradAcc<NV> A;
        for (int32_t k = g.xptr[r] + lane; k < g.xptr[r + 1]; k += 64) {
            const int64_t j = g.xidx[k];
            const double ex = g.x[j] - xi, ey = g.y[j] - yi;
            const double l2 = ex * ex + ey * ey;
            double rr = __builtin_amdgcn_rsq(l2);
            rr = rr * __builtin_fma(-0.5 * l2 * rr, rr, 1.5);
            const double r3 = rr * rr * rr;
            const double wx = ex * r3, wy = ey * r3;
            A.q0 = __builtin_fma(ex, wx, A.q0);
            A.q1 = __builtin_fma(ex, wy, A.q1);
            A.q3 = __builtin_fma(ey, wy, A.q3);
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const double gx = gin ? gin[2 * (v * n + j)] : 0.0, gy = gin ? gin[2 * (v * n + j) + 1] : 0.0;
                const double df2 = -ex * gx - ey * gy;
                const double w = 6 * (fi[v] - f[v * n + j]) - 2 * df2;
                A.s0[v] = __builtin_fma(w, wx, A.s0[v]);
                A.s1[v] = __builtin_fma(w, wy, A.s1[v]);
            }
        }
        for (int off = 32; off > 0; off >>= 1) {
            A.q0 += __shfl_down(A.q0, off);
            A.q1 += __shfl_down(A.q1, off);
            A.q3 += __shfl_down(A.q3, off);
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                A.s0[v] += __shfl_down(A.s0[v], off);
                A.s1[v] += __shfl_down(A.s1[v], off);
            }
        }
        if (lane == 0) {
            double* d = out + r * (3 + 2 * NV);
            d[0] = A.q0;
            d[1] = A.q1;
            d[2] = A.q3;
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                d[3 + 2 * v] = A.s0[v];
                d[4 + 2 * v] = A.s1[v];
            }
        }
    }
}

// ------------------------------------------------------------------ cone solve (fixed K sweeps)
//
// After K Chebyshev sweeps from x_0 = 0 a vertex's gradient depends only on the vertices within K
// hops of it (each sweep reads the 1-hop neighbours' previous iterate and the vertex's own
// iterate before that). The interpolated values need the gradients at the vertices of the
// triangles that hold targets only, so for a 128^2 target grid over a 1e7-point lattice the global
// iteration's x_K there is formed from small patches instead of K passes over the whole lattice:
//   * interior targets (their cell more than K + 1 cells from the lattice boundary): one workgroup
//     per target cell holds the (2K + 4)^2 box around the cell in LDS and runs the K sweeps on the
//     shrinking square that still influences the cell (x_j on the vertices within K + 1 - j of it);
//   * the rest (cells near the boundary, pocket triangles): the ring's pocket chords couple vertices
//     far along a side, so those run the global iteration on the boundary band (depth <= 2K + 3 - j
//     at sweep j, one launch per sweep, the chords in the ring kernel), valid to depth K + 3 after K
//     sweeps.
// Per vertex the edge order and arithmetic are k_gd_grad's / k_gd_grad_ring's, so the result at
// every target vertex is the global iteration's K-sweep value bit for bit
// (tests/test_gpu_parity.py::test_gradient_cone_equals_global_sweeps).

constexpr int kClaimAxisLds = 512;                // target axes up to this long go to LDS in k_gd_claim_hit
constexpr int kConeMaxK = 14;                    // patch box side 2K + 4 <= 32
constexpr int kConeBox = 2 * kConeMaxK + 4;

// grad_edge on values: neighbour (xj, yj), its values fj and previous gradients (gxj, gyj)
template <int NV>
__device__ __forceinline__ void edge_vals(double xj, double yj, const double (&fj)[NV], const double (&gxj)[NV],
                                          const double (&gyj)[NV], double xi, double yi, const double (&fi)[NV],
                                          GradAcc<NV>& A) {
    const double ex = xj - xi, ey = yj - yi;
    const double l2 = ex * ex + ey * ey;
    double r = __builtin_amdgcn_rsq(l2);
    r = r * __builtin_fma(-0.5 * l2 * r, r, 1.5);
    const double r3 = r * r * r;
    const double wx = ex * r3, wy = ey * r3;
    A.q0 = __builtin_fma(ex, wx, A.q0);
    A.q1 = __builtin_fma(ex, wy, A.q1);
    A.q3 = __builtin_fma(ey, wy, A.q3);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const double df2 = -ex * gxj[v] - ey * gyj[v];
        const double w = 6 * (fi[v] - fj[v]) - 2 * df2;
        A.s0[v] = __builtin_fma(w, wx, A.s0[v]);
        A.s1[v] = __builtin_fma(w, wy, A.s1[v]);
    }
}

// sweep j's weight and predecessor form: j = 1 plain, j = 2 against x_0 = 0, later against x_{j-2}
struct ConeStep {
    int mode;  // 0 plain, 1 zero predecessor, 2 predecessor x_{j-2}
    double omega;
};

// grad_solve on values: returns scipy's change measure; (ox, oy) = the new gradient
template <int NV>
__device__ __forceinline__ double solve_vals(const GradAcc<NV>& A, int v, double gix, double giy, const ConeStep& st,
                                             double px, double py, double& ox, double& oy) {
    const double q0 = 4 * A.q0, q1 = 4 * A.q1, q3 = 4 * A.q3;
    const double inv = 1.0 / (q0 * q3 - q1 * q1);
    const double r0 = (q3 * A.s0[v] - q1 * A.s1[v]) * inv;
    const double r1 = (-q1 * A.s0[v] + q0 * A.s1[v]) * inv;
    const double c = fmax(fabs(gix + r0), fabs(giy + r1)) / fmax(1.0, fmax(fabs(r0), fabs(r1)));
    if (st.mode == 2) {
        ox = st.omega * (-r0 - px) + px;
        oy = st.omega * (-r1 - py) + py;
    } else if (st.mode == 1) {
        ox = st.omega * (-r0 - 0.0) + 0.0;
        oy = st.omega * (-r1 - 0.0) + 0.0;
    } else {
        ox = -r0;
        oy = -r1;
    }
    return c;
}

// the boundary band: vertices with min(iv, ih, nv - 1 - iv, nh - 1 - ih) <= D, enumerated as the
// top rows, the bottom rows, then the left / right column pieces of the rows between
struct BandMap {
    int nv, nh, D;
    int rows_top, rows_bot, mid0, mid1, cols;  // full rows [0, rows_top), [nv - rows_bot, nv); side columns
    int64_t n_top, n_bot, n_mid, total;
};

inline BandMap band_map(int nv, int nh, int D) {
    BandMap b{nv, nh, D, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    b.rows_top = std::min(D + 1, nv);
    b.rows_bot = std::min(D + 1, nv - b.rows_top);
    b.mid0 = b.rows_top;
    b.mid1 = nv - b.rows_bot;
    b.cols = std::min(D + 1, nh / 2);
    const bool full_mid = 2 * (D + 1) >= nh;
    b.n_top = (int64_t)b.rows_top * nh;
    b.n_bot = (int64_t)b.rows_bot * nh;
    b.n_mid = (int64_t)(b.mid1 - b.mid0) * (full_mid ? nh : 2 * b.cols);
    if (full_mid) b.cols = -1;
    b.total = b.n_top + b.n_bot + b.n_mid;
    return b;
}

__device__ __forceinline__ int64_t band_vertex(const BandMap& b, int64_t k) {
    if (k < b.n_top) return k;
    k -= b.n_top;
    if (k < b.n_bot) return (int64_t)(b.nv - b.rows_bot) * b.nh + k;
    k -= b.n_bot;
    if (b.cols < 0) return (int64_t)b.mid0 * b.nh + k;
    const int w = 2 * b.cols;
    const int r = b.mid0 + (int)(k / w), c = (int)(k - (int64_t)(k / w) * w);
    return (int64_t)r * b.nh + (c < b.cols ? c : b.nh - 2 * b.cols + c);
}

template <int NV>
struct ConeBand {
    const double* f;   // (NV, n)
    const double* gin;    // x_{j-1} (NV, n, 2) or nullptr (x_0 = 0)
    const double* gprev;  // x_{j-2} (mode 2)
    double* gout;         // x_j
    double* ring_acc;     // (L, 3 + 2 NV): ring vertices' grid-edge sums, solved by k_gd_cone_ring
    ConeStep st;
    const int* needed;    // device flag: some target needs the band (else the launch returns at once)
};

// vertex i's lattice-edge sums of one band sweep (k_gd_grad's edge order: left, right, down, up,
// then the diagonals present)
template <int NV>
__device__ __forceinline__ void band_grid_sums(const Grid& g, const ConeBand<NV>& a, int64_t n, int64_t i, int iv,
                                               int ih, double xi, double yi, const double (&fi)[NV],
                                               GradAcc<NV>& A) {
    if constexpr (NV == 1) {
        // every candidate neighbour's data loaded first (positions off the lattice clamped to i,
        // the diagonals' presence from their cells' bytes, loaded beside them), then the edges in
        // the same order and arithmetic: one memory round trip per vertex instead of one per edge
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
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (on[k]) {
                const double fj[1] = {fs[k]}, gxj[1] = {gxs[k]}, gyj[1] = {gys[k]};
                edge_vals<1>(xs[k], ys[k], fj, gxj, gyj, xi, yi, fi, A);
            }
        return;
    }
    auto edge = [&](int64_t j) {
        double fj[NV], gxj[NV], gyj[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            fj[v] = a.f[v * n + j];
            gxj[v] = a.gin ? a.gin[2 * (v * n + j)] : 0.0;
            gyj[v] = a.gin ? a.gin[2 * (v * n + j) + 1] : 0.0;
        }
        edge_vals<NV>(g.x[j], g.y[j], fj, gxj, gyj, xi, yi, fi, A);
    };
    if (ih > 0) edge(i - 1);
    if (ih < g.nh - 1) edge(i + 1);
    if (iv > 0) edge(i - g.nh);
    if (iv < g.nv - 1) edge(i + g.nh);
    const int64_t c0 = (int64_t)iv * (g.nh - 1) + ih;
    if (iv > 0 && ih > 0 && g.diag[c0 - g.nh] == 0) edge(i - g.nh - 1);
    if (iv > 0 && ih < g.nh - 1 && g.diag[c0 - (g.nh - 1)] == 1) edge(i - g.nh + 1);
    if (iv < g.nv - 1 && ih > 0 && g.diag[c0 - 1] == 1) edge(i + g.nh - 1);
    if (iv < g.nv - 1 && ih < g.nh - 1 && g.diag[c0] == 0) edge(i + g.nh + 1);
}

// one sweep of the band (k_gd_grad's per-vertex body; nothing reads outside the lattice)
template <int NV>
__global__ void __launch_bounds__(kBlock) k_gd_cone_band(Grid g, BandMap bm, ConeBand<NV> a) {
    if (!*a.needed) return;
    const int64_t n = (int64_t)g.nv * g.nh;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < bm.total;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = band_vertex(bm, k);
        const int iv = (int)(i / g.nh), ih = (int)(i - (int64_t)iv * g.nh);
        const double xi = g.x[i], yi = g.y[i];
        double fi[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) fi[v] = a.f[v * n + i];
        GradAcc<NV> A;
        band_grid_sums<NV>(g, a, n, i, iv, ih, xi, yi, fi, A);
        const int64_t r = ring_pos(g, iv, ih);
        if (r >= 0) {
            double* d = a.ring_acc + r * (3 + 2 * NV);
            d[0] = A.q0;
            d[1] = A.q1;
            d[2] = A.q3;
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                d[3 + 2 * v] = A.s0[v];
                d[4 + 2 * v] = A.s1[v];
            }
            continue;
        }
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const int64_t o = 2 * (v * n + i);
            const double gix = a.gin ? a.gin[o] : 0.0, giy = a.gin ? a.gin[o + 1] : 0.0;
            const double px = a.st.mode == 2 ? a.gprev[o] : 0.0, py = a.st.mode == 2 ? a.gprev[o + 1] : 0.0;
            double ox, oy;
            solve_vals<NV>(A, v, gix, giy, a.st, px, py, ox, oy);
            a.gout[o] = ox;
            a.gout[o + 1] = oy;
        }
    }
}

// the ring vertices of a band sweep: pocket chords (a wave per ring vertex, k_gd_grad_ring's fixed
// reduction order), then the grid-edge sums the band kernel left, then the solve
// ring vertex r's lattice index (the ring in k_gd_grad_ring's order)
__device__ __forceinline__ int64_t ring_vertex(const Grid& g, int64_t r) {
    const int64_t ra = g.nh - 1, rb = g.nv - 1;
    if (r < ra) return r;
    if (r < ra + rb) return (r - ra) * g.nh + (g.nh - 1);
    if (r < 2 * ra + rb) return (int64_t)(g.nv - 1) * g.nh + (g.nh - 1 - (r - ra - rb));
    return (int64_t)(g.nv - 1 - (r - 2 * ra - rb)) * g.nh;
}

// ring vertex r's pocket chords (one per lane of a group of W lanes, W >= the chord count, or
// strided over a whole wave), reduced over the group by the butterfly k_gd_grad_ring uses over a
// wave, then (lead lane) the band kernel's grid-edge sums added and the solve. For a count <= W the
// W-lane tree is the 64-lane tree with its zero partners left out: the same bits.
template <int NV, int W, bool GRID = false>
__device__ __forceinline__ void cone_ring_vertex(const Grid& g, const ConeBand<NV>& a, int64_t r, int sub) {
    const int64_t n = (int64_t)g.nv * g.nh;
    const int64_t i = ring_vertex(g, r);
    const double xi = g.x[i], yi = g.y[i];
    double fi[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) fi[v] = a.f[v * n + i];
    GradAcc<NV> D;  // GRID: the lattice-edge sums, formed here by the lead lane (else the band kernel's)
    if (GRID && sub == 0) {
        const int iv = (int)(i / g.nh), ih = (int)(i - (int64_t)iv * g.nh);
        band_grid_sums<NV>(g, a, n, i, iv, ih, xi, yi, fi, D);
    }
    GradAcc<NV> A;
    for (int32_t k = g.xptr[r] + sub; k < g.xptr[r + 1]; k += W) {
        const int64_t j = g.xidx[k];
        double fj[NV], gxj[NV], gyj[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            fj[v] = a.f[v * n + j];
            gxj[v] = a.gin ? a.gin[2 * (v * n + j)] : 0.0;
            gyj[v] = a.gin ? a.gin[2 * (v * n + j) + 1] : 0.0;
        }
        edge_vals<NV>(g.x[j], g.y[j], fj, gxj, gyj, xi, yi, fi, A);
    }
    for (int off = W / 2; off > 0; off >>= 1) {
        A.q0 += __shfl_down(A.q0, off, W);
        A.q1 += __shfl_down(A.q1, off, W);
        A.q3 += __shfl_down(A.q3, off, W);
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            A.s0[v] += __shfl_down(A.s0[v], off, W);
            A.s1[v] += __shfl_down(A.s1[v], off, W);
        }
    }
    if (sub == 0) {
        if (GRID) {
            A.q0 += D.q0;
            A.q1 += D.q1;
            A.q3 += D.q3;
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                A.s0[v] += D.s0[v];
                A.s1[v] += D.s1[v];
            }
        } else {
            const double* d = a.ring_acc + r * (3 + 2 * NV);
            A.q0 += d[0];
            A.q1 += d[1];
            A.q3 += d[2];
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                A.s0[v] += d[3 + 2 * v];
                A.s1[v] += d[4 + 2 * v];
            }
        }
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const int64_t o = 2 * (v * n + i);
            const double gix = a.gin ? a.gin[o] : 0.0, giy = a.gin ? a.gin[o + 1] : 0.0;
            const double px = a.st.mode == 2 ? a.gprev[o] : 0.0, py = a.st.mode == 2 ? a.gprev[o + 1] : 0.0;
            double ox, oy;
            solve_vals<NV>(A, v, gix, giy, a.st, px, py, ox, oy);
            a.gout[o] = ox;
            a.gout[o + 1] = oy;
        }
    }
}

// the ring's solve for one sweep: eight ring vertices per wave, eight lanes each (a ring vertex
// has a few pocket chords); a vertex with more than eight takes the whole wave afterwards
// (k_gd_grad_ring's 64-lane loop and tree). Either way its bits are k_gd_grad_ring's.
template <int NV>
__global__ void __launch_bounds__(kBlock) k_gd_cone_ring(Grid g, ConeBand<NV> a) {
    if (!*a.needed) return;
    const int64_t L = 2 * (int64_t)(g.nh - 1) + 2 * (int64_t)(g.nv - 1);
    const int lane = threadIdx.x & 63, sub = lane & 7;
    for (int64_t r0 = ((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6) * 8; r0 < L;
         r0 += (((int64_t)gridDim.x * blockDim.x) >> 6) * 8) {
        const int64_t r = r0 + (lane >> 3);
        const bool big = r < L && g.xptr[r + 1] - g.xptr[r] > 8;
        if (r < L && !big) cone_ring_vertex<NV, 8>(g, a, r, sub);
        unsigned long long m = __ballot(big && sub == 0);
        while (m) {  // wave-uniform
            const int q = __builtin_ctzll(m);
            m &= m - 1;
            cone_ring_vertex<NV, 64>(g, a, r0 + (q >> 3), lane);
        }
    }
}

// one sweep of the band in one launch, the ring in 8-lane groups: workgroups [0, nbw) take the band's
// vertices off the ring (k_gd_cone_band's body), the rest eight ring vertices per wave - the lead
// lane forms the vertex's lattice-edge sums itself (band_grid_sums, what k_gd_cone_band would have
// left in ring_acc), the chords as k_gd_cone_ring. Both halves read x_{j-1} / x_{j-2} only: the
// two-launch form's bits in one launch per sweep.
template <int NV>
__global__ void __launch_bounds__(kBlock) k_gd_cone_sweep8(Grid g, BandMap bm, ConeBand<NV> a, int nbw) {
    if (!*a.needed) return;
    const int64_t n = (int64_t)g.nv * g.nh;
    if ((int)blockIdx.x < nbw) {
        for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < bm.total;
             k += (int64_t)nbw * blockDim.x) {
            const int64_t i = band_vertex(bm, k);
            const int iv = (int)(i / g.nh), ih = (int)(i - (int64_t)iv * g.nh);
            if (ring_pos(g, iv, ih) >= 0) continue;
            const double xi = g.x[i], yi = g.y[i];
            double fi[NV];
#pragma unroll
            for (int v = 0; v < NV; ++v) fi[v] = a.f[v * n + i];
            GradAcc<NV> A;
            band_grid_sums<NV>(g, a, n, i, iv, ih, xi, yi, fi, A);
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const int64_t o = 2 * (v * n + i);
                const double gix = a.gin ? a.gin[o] : 0.0, giy = a.gin ? a.gin[o + 1] : 0.0;
                const double px = a.st.mode == 2 ? a.gprev[o] : 0.0, py = a.st.mode == 2 ? a.gprev[o + 1] : 0.0;
                double ox, oy;
                solve_vals<NV>(A, v, gix, giy, a.st, px, py, ox, oy);
                a.gout[o] = ox;
                a.gout[o + 1] = oy;
            }
        }
        return;
    }
    const int64_t L = 2 * (int64_t)(g.nh - 1) + 2 * (int64_t)(g.nv - 1);
    const int lane = threadIdx.x & 63, sub = lane & 7;
    const int64_t w0 = ((int64_t)(blockIdx.x - nbw) * blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)(gridDim.x - nbw) * blockDim.x) >> 6;
    for (int64_t r0 = w0 * 8; r0 < L; r0 += nw * 8) {
        const int64_t r = r0 + (lane >> 3);
        const bool big = r < L && g.xptr[r + 1] - g.xptr[r] > 8;
        if (r < L && !big) cone_ring_vertex<NV, 8, true>(g, a, r, sub);
        unsigned long long m = __ballot(big && sub == 0);
        while (m) {  // wave-uniform
            const int q = __builtin_ctzll(m);
            m &= m - 1;
            cone_ring_vertex<NV, 64, true>(g, a, r0 + (q >> 3), lane);
        }
    }
}

// one sweep of the band in one launch: the band's vertices off the ring (k_gd_cone_band's body) in
// the first `nb` workgroups, then a wave per ring vertex - the pocket chords reduced over the
// wave, then the vertex's grid edges (lane 0, k_gd_cone_band's order), added to the chord sums in
// that order as k_gd_cone_ring adds the band kernel's partial sums - then the solve. Both halves
// read x_{j-1} / x_{j-2} only, so one launch per sweep gives k_gd_cone_band + k_gd_cone_ring's bits.
template <int NV>
__global__ void __launch_bounds__(kBlock) k_gd_cone_sweep(Grid g, BandMap bm, ConeBand<NV> a, int nbw) {
    if (!*a.needed) return;
    const int64_t n = (int64_t)g.nv * g.nh;
    // the grid-edge sums of vertex i (k_gd_cone_band's edge order)
    auto grid_sums = [&](int64_t i, int iv, int ih, double xi, double yi, const double (&fi)[NV], GradAcc<NV>& A) {
        auto edge = [&](int64_t j) {
            double fj[NV], gxj[NV], gyj[NV];
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                fj[v] = a.f[v * n + j];
                gxj[v] = a.gin ? a.gin[2 * (v * n + j)] : 0.0;
                gyj[v] = a.gin ? a.gin[2 * (v * n + j) + 1] : 0.0;
            }
            edge_vals<NV>(g.x[j], g.y[j], fj, gxj, gyj, xi, yi, fi, A);
        };
        if (ih > 0) edge(i - 1);
        if (ih < g.nh - 1) edge(i + 1);
        if (iv > 0) edge(i - g.nh);
        if (iv < g.nv - 1) edge(i + g.nh);
        const int64_t c0 = (int64_t)iv * (g.nh - 1) + ih;
        if (iv > 0 && ih > 0 && g.diag[c0 - g.nh] == 0) edge(i - g.nh - 1);
        if (iv > 0 && ih < g.nh - 1 && g.diag[c0 - (g.nh - 1)] == 1) edge(i - g.nh + 1);
        if (iv < g.nv - 1 && ih > 0 && g.diag[c0 - 1] == 1) edge(i + g.nh - 1);
        if (iv < g.nv - 1 && ih < g.nh - 1 && g.diag[c0] == 0) edge(i + g.nh + 1);
    };
    auto solve_store = [&](int64_t i, const GradAcc<NV>& A) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const int64_t o = 2 * (v * n + i);
            const double gix = a.gin ? a.gin[o] : 0.0, giy = a.gin ? a.gin[o + 1] : 0.0;
            const double px = a.st.mode == 2 ? a.gprev[o] : 0.0, py = a.st.mode == 2 ? a.gprev[o + 1] : 0.0;
            double ox, oy;
            solve_vals<NV>(A, v, gix, giy, a.st, px, py, ox, oy);
            a.gout[o] = ox;
            a.gout[o + 1] = oy;
        }
    };
    if ((int)blockIdx.x < nbw) {
        for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < bm.total; k += (int64_t)nbw * blockDim.x) {
            const int64_t i = band_vertex(bm, k);
            const int iv = (int)(i / g.nh), ih = (int)(i - (int64_t)iv * g.nh);
            if (ring_pos(g, iv, ih) >= 0) continue;  // the ring's waves below
            const double xi = g.x[i], yi = g.y[i];
            double fi[NV];
#pragma unroll
            for (int v = 0; v < NV; ++v) fi[v] = a.f[v * n + i];
            GradAcc<NV> A;
            grid_sums(i, iv, ih, xi, yi, fi, A);
            solve_store(i, A);
        }
        return;
    }
    const int64_t ra = g.nh - 1, rb = g.nv - 1, L = 2 * ra + 2 * rb;
    const int lane = threadIdx.x & 63;
    const int64_t nwave = ((int64_t)(gridDim.x - nbw) * blockDim.x) >> 6;
    for (int64_t r = (((int64_t)blockIdx.x - nbw) * blockDim.x + threadIdx.x) >> 6; r < L; r += nwave) {
        int64_t i;
        if (r < ra) i = r;
        else if (r < ra + rb) i = (r - ra) * g.nh + (g.nh - 1);
        else if (r < 2 * ra + rb) i = (int64_t)(g.nv - 1) * g.nh + (g.nh - 1 - (r - ra - rb));
        else i = (int64_t)(g.nv - 1 - (r - 2 * ra - rb)) * g.nh;
        const double xi = g.x[i], yi = g.y[i];
        double fi[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) fi[v] = a.f[v * n + i];
        GradAcc<NV> A;
        for (int32_t k = g.xptr[r] + lane; k < g.xptr[r + 1]; k += 64) {
            const int64_t j = g.xidx[k];
            double fj[NV], gxj[NV], gyj[NV];
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                fj[v] = a.f[v * n + j];
                gxj[v] = a.gin ? a.gin[2 * (v * n + j)] : 0.0;
                gyj[v] = a.gin ? a.gin[2 * (v * n + j) + 1] : 0.0;
            }
            edge_vals<NV>(g.x[j], g.y[j], fj, gxj, gyj, xi, yi, fi, A);
        }
        for (int off = 32; off > 0; off >>= 1) {
            A.q0 += __shfl_down(A.q0, off);
            A.q1 += __shfl_down(A.q1, off);
            A.q3 += __shfl_down(A.q3, off);
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                A.s0[v] += __shfl_down(A.s0[v], off);
                A.s1[v] += __shfl_down(A.s1[v], off);
            }
        }
        if (lane == 0) {
            const int iv = (int)(i / g.nh), ih = (int)(i - (int64_t)iv * g.nh);
            GradAcc<NV> G;
            grid_sums(i, iv, ih, xi, yi, fi, G);
            A.q0 += G.q0;
            A.q1 += G.q1;
            A.q3 += G.q3;
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                A.s0[v] += G.s0[v];
                A.s1[v] += G.s1[v];
            }
            solve_store(i, A);
        }
    }
}

template <int NV>
struct ConePatch {
    const double* f;           // (NV, n)
    const int64_t* cells;      // interior target cells (duplicates allowed)
    const int* count;          // how many (device)
    int K;
    ConeStep st[kConeMaxK + 1];  // st[j] for sweep j = 1 .. K
    double* gout;              // x_K (NV, n, 2): the cells' four corners are written
    unsigned long long* chg;   // largest change measure of one more sweep at the corners (or nullptr)
    unsigned long long* clk;   // diagnostics (AKB_GD_PATCH_CLOCK): cycles per phase summed over cells, or nullptr
};

// one workgroup per interior target cell: the (2K + 4)^2 box around it in LDS, K sweeps on the
// shrinking square that influences the cell, the corners' x_K to global memory
template <int NV>
__global__ void __launch_bounds__(256) k_gd_cone_patch(Grid g, ConePatch<NV> a) {
    constexpr int B2 = kConeBox * kConeBox;
    __shared__ double sx[B2], sy[B2], sf[NV][B2];
    __shared__ double sg[3][NV][B2][2];  // x_{j-2}, x_{j-1}, x_j rotating
    __shared__ uint8_t sd[B2];
    const int64_t n = (int64_t)g.nv * g.nh;
    const int K = a.K, W = 2 * K + 4;
    for (int pid = blockIdx.x; pid < *a.count; pid += gridDim.x) {
        const int64_t cell = a.cells[pid];
        const int iv0 = (int)(cell / (g.nh - 1)), ih0 = (int)(cell - (int64_t)iv0 * (g.nh - 1));
        const int R0 = iv0 - (K + 1), C0 = ih0 - (K + 1);
        __syncthreads();  // the previous cell's reads are done
        for (int idx = threadIdx.x; idx < W * W; idx += blockDim.x) {
            const int r = idx / W, c = idx - (idx / W) * W;
            const int64_t i = (int64_t)(R0 + r) * g.nh + (C0 + c);
            sx[idx] = g.x[i];
            sy[idx] = g.y[i];
#pragma unroll
            for (int v = 0; v < NV; ++v) sf[v][idx] = a.f[v * n + i];
            sd[idx] = (r < W - 1 && c < W - 1) ? g.diag[(int64_t)(R0 + r) * (g.nh - 1) + (C0 + c)] : 0;
        }
        __syncthreads();
        // the sums of box vertex b from iterate buffer `in` (nullptr role: x_0 = 0)
        auto sums = [&](int b, int in) {
            GradAcc<NV> A;
            double fi[NV];
#pragma unroll
            for (int v = 0; v < NV; ++v) fi[v] = sf[v][b];
            const double xi = sx[b], yi = sy[b];
            auto edge = [&](int j) {
                double fj[NV], gxj[NV], gyj[NV];
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    fj[v] = sf[v][j];
                    gxj[v] = in < 0 ? 0.0 : sg[in][v][j][0];
                    gyj[v] = in < 0 ? 0.0 : sg[in][v][j][1];
                }
                edge_vals<NV>(sx[j], sy[j], fj, gxj, gyj, xi, yi, fi, A);
            };
            // k_gd_grad's order: left, right, down (iv - 1), up (iv + 1), then the diagonals
            edge(b - 1);
            edge(b + 1);
            edge(b - W);
            edge(b + W);
            if (sd[b - W - 1] == 0) edge(b - W - 1);
            if (sd[b - W] == 1) edge(b - W + 1);
            if (sd[b - 1] == 1) edge(b + W - 1);
            if (sd[b] == 0) edge(b + W + 1);
            return A;
        };
        for (int j = 1; j <= K; ++j) {
            const int half = K + 1 - j, side = 2 * half + 2, off = (K + 1) - half;
            const int in = j == 1 ? -1 : (j - 1) % 3, out = j % 3, prev = (j + 1) % 3;  // x_{j-1}, x_j, x_{j-2}
            const ConeStep st = a.st[j];
            for (int idx = threadIdx.x; idx < side * side; idx += blockDim.x) {
                const int b = (off + idx / side) * W + off + (idx - (idx / side) * side);
                const GradAcc<NV> A = sums(b, in);
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    const double gix = in < 0 ? 0.0 : sg[in][v][b][0], giy = in < 0 ? 0.0 : sg[in][v][b][1];
                    const double px = st.mode == 2 ? sg[prev][v][b][0] : 0.0;
                    const double py = st.mode == 2 ? sg[prev][v][b][1] : 0.0;
                    double ox, oy;
                    solve_vals<NV>(A, v, gix, giy, st, px, py, ox, oy);
                    sg[out][v][b][0] = ox;
                    sg[out][v][b][1] = oy;
                }
            }
            __syncthreads();
        }
        // the cell's corners: x_K out, and the change one more (plain-measured) sweep would make
        double worst = 0.0;
        if (threadIdx.x < 4) {
            const int cr = K + 1 + (threadIdx.x >> 1), cc = K + 1 + (threadIdx.x & 1);
            const int b = cr * W + cc, fin = K % 3;
            const int64_t i = (int64_t)(R0 + cr) * g.nh + (C0 + cc);
            const GradAcc<NV> A = sums(b, fin);
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const double gx = sg[fin][v][b][0], gy = sg[fin][v][b][1];
                a.gout[2 * (v * n + i)] = gx;
                a.gout[2 * (v * n + i) + 1] = gy;
                double ox, oy;
                worst = fmax(worst, solve_vals<NV>(A, v, gx, gy, ConeStep{0, 1.0}, 0.0, 0.0, ox, oy));
            }
        }
        if (a.chg && threadIdx.x < 64) {
            for (int off = 2; off > 0; off >>= 1) worst = fmax(worst, __shfl_down(worst, off));
            if (threadIdx.x == 0 && worst > 0) atomicMax(a.chg, (unsigned long long)__double_as_longlong(worst));
        }
    }
}

// k_gd_cone_patch with one thread per box vertex (one value set): the edge geometry of a vertex -
// (ex, ey), r^-3 and 6 (f_i - f_j) per edge, the local 2 x 2 system and its reciprocal
// determinant - does not change between sweeps, so each thread forms its own once per cell, in
// k_gd_grad's expressions and edge order, and keeps it in registers; a sweep then costs per edge
// one LDS read of the neighbour's iterate and nine operations (against the full edge_vals: a
// reciprocal square root and ~25 operations, five LDS reads). The box has pitch 32; threads take
// its vertices in order of depth; x_j overwrites x_{j-2} in place (a vertex reads its own predecessor only),
// so two iterate buffers suffice. The arithmetic is edge_vals / solve_vals' exactly: x_K at the
// corners equals k_gd_cone_patch's, bit for bit.
template <bool PF, bool CLK>
__global__ void __launch_bounds__(1024) k_gd_cone_patch1(Grid g, ConePatch<1> a, int rowmajor) {
    constexpr int P = 33;  // LDS pitch: a column of the box steps 2 banks per row, not 0
    static_assert(kConeBox < P, "box pitch");
    __shared__ double sxyf[2][3][P * 32];  // x, y, f of the box; two sets (PF: the next cell's DMA)
    __shared__ double2 sg[2][P * 32];
    __shared__ uint8_t sd[P * 32];
    const int K = a.K, W = 2 * K + 4;
    const int t = threadIdx.x;
    // this thread's vertex, in order of depth from the box's centre outwards: vertex (r, c) of depth
    // d = min(r, c, W-1-r, W-1-c) takes part in sweeps 1 .. d, so sweep j's vertices are a prefix of
    // the threads - its waves are full, the rest idle (row-major lanes would run each sweep's
    // shrinking square at ~half occupancy). The four innermost are the cell's corners.
    int r = -1, c = -1, dep = 0;
    if (rowmajor) {  // A/B: lanes along the box's rows
        r = t / 32;
        c = t - (t / 32) * 32;
        dep = (r < W && c < W) ? min(min(r, c), min(W - 1 - r, W - 1 - c)) : 0;
        if (dep > K + 1) dep = K + 1;
    } else {
        int rem = t;
        for (int d = W / 2 - 1; d >= 1; --d) {
            const int s1 = W - 2 * d - 1, cnt = 4 * s1;
            if (rem < cnt) {
                if (rem < s1) { r = d; c = d + rem; }
                else if (rem < 2 * s1) { r = d + (rem - s1); c = d + s1; }
                else if (rem < 3 * s1) { r = d + s1; c = d + s1 - (rem - 2 * s1); }
                else { r = d + s1 - (rem - 3 * s1); c = d; }
                dep = d;
                break;
            }
            rem -= cnt;
        }
    }
    const bool mine = dep >= 1;
    const int b = mine ? r * P + c : 0;
    // the box load. PF: one persistent workgroup walks its cells; x, y, f of the next cell go
    // global -> LDS by DMA (global_load_lds, no registers) into the other set while this cell's
    // sweeps run - one wave instruction per box row and array, lane i moving dword i of the row.
    // The diagonal bytes go through a register (one per thread, row-major). Else everything
    // through registers, row-major (coalesced), at the top of the cell.
    const int count = *a.count;
    const double* const gx_ = g.x;
    const double* const gy_ = g.y;
    const double* const gf_ = a.f;
    const uint8_t* const gd_ = g.diag;
    const int nh = g.nh;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
    const int lr = t / 32, lc = t - (t / 32) * 32;
    // the next cell's box: the diagonal byte into a register, then x, y, f by DMA (issued after every
    // load the wave waits on, so no wait before the next cell's top lands on them)
    auto prefetch = [=](int pid, int st, uint8_t& d) {
        if (pid >= count) return;
        const int64_t cell = a.cells[pid];
        const int iv0 = (int)(cell / (nh - 1)), ih0 = (int)(cell - (int64_t)iv0 * (nh - 1));
        const int R0 = iv0 - (K + 1), C0 = ih0 - (K + 1);
        if (lr < W - 1 && lc < W - 1) d = gd_[(int64_t)(R0 + lr) * (nh - 1) + (C0 + lc)];
#pragma unroll
        for (int arr = 0; arr < 3; ++arr) {
            const double* base = arr == 0 ? gx_ : arr == 1 ? gy_ : gf_;
            for (int row = wv; row < W; row += 16) {
                const double* src = base + (int64_t)(R0 + row) * nh + C0;
                if (lane < 2 * W)
                    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) const char*)src + lane * 4,
                                                     (__attribute__((address_space(3))) void*)&sxyf[st][arr][row * P],
                                                     4, 0, 0);
            }
        }
    };
    uint8_t pd = 0;
    if (PF) prefetch(blockIdx.x, 0, pd);
    double cmax = 0.0;  // the corners' change measure over this workgroup's cells: one atomic at the end
    int set = 0;
    for (int pid = blockIdx.x; pid < count; pid += gridDim.x, set ^= (PF ? 1 : 0)) {
        const int64_t cell = a.cells[pid];
        const int iv0 = (int)(cell / (g.nh - 1)), ih0 = (int)(cell - (int64_t)iv0 * (g.nh - 1));
        const int R0 = iv0 - (K + 1), C0 = ih0 - (K + 1);
        const unsigned long long c0 = CLK ? clock64() : 0;
        double* const sx = sxyf[set][0];
        double* const sy = sxyf[set][1];
        double* const sf = sxyf[set][2];
        {
            double nx_ = 0.0, ny_ = 0.0, nf_ = 0.0;
            uint8_t nd_ = pd;
            if (!PF && lr < W && lc < W) {
                const int64_t i = (int64_t)(R0 + lr) * nh + (C0 + lc);
                nx_ = gx_[i];
                ny_ = gy_[i];
                nf_ = gf_[i];
                nd_ = (lr < W - 1 && lc < W - 1) ? gd_[(int64_t)(R0 + lr) * (nh - 1) + (C0 + lc)] : 0;
            }
            if (PF) __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA rows have landed (vmcnt)
            __syncthreads();  // the previous cell's reads are done; PF: every wave's DMA has landed
            if (lr < W && lc < W) {
                const int q = lr * P + lc;
                if (!PF) {
                    sx[q] = nx_;
                    sy[q] = ny_;
                    sf[q] = nf_;
                }
                sd[q] = nd_;
            }
        }
        __syncthreads();
        const unsigned long long c1 = CLK ? clock64() : 0;
        if (PF) {
            pd = 0;
            prefetch(pid + gridDim.x, set ^ 1, pd);
        }
        // this vertex's edges in k_gd_grad's order: left, right, down, up, then the diagonals
        int nb[8];
        unsigned em = 0;
        double ex[8], ey[8], r3[8], c6[8];
        double q0 = 0.0, q1 = 0.0, q3 = 0.0, inv = 0.0;
        if (mine) {
            nb[0] = b - 1;
            nb[1] = b + 1;
            nb[2] = b - P;
            nb[3] = b + P;
            nb[4] = b - P - 1;
            nb[5] = b - P + 1;
            nb[6] = b + P - 1;
            nb[7] = b + P + 1;
            em = 0x0fu | (sd[b - P - 1] == 0 ? 0x10u : 0u) | (sd[b - P] == 1 ? 0x20u : 0u) |
                 (sd[b - 1] == 1 ? 0x40u : 0u) | (sd[b] == 0 ? 0x80u : 0u);
            const double xi = sx[b], yi = sy[b], fi = sf[b];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                ex[k] = ey[k] = r3[k] = c6[k] = 0.0;
                if (!(em & (1u << k))) continue;
                const int j = nb[k];
                const double exk = sx[j] - xi, eyk = sy[j] - yi;
                const double l2 = exk * exk + eyk * eyk;
                double rr = __builtin_amdgcn_rsq(l2);
                rr = rr * __builtin_fma(-0.5 * l2 * rr, rr, 1.5);
                const double r3k = rr * rr * rr;
                const double wx = exk * r3k, wy = eyk * r3k;
                q0 = __builtin_fma(exk, wx, q0);
                q1 = __builtin_fma(exk, wy, q1);
                q3 = __builtin_fma(eyk, wy, q3);
                ex[k] = exk;
                ey[k] = eyk;
                r3[k] = r3k;
                c6[k] = 6 * (fi - sf[j]);
            }
            q0 = 4 * q0;
            q1 = 4 * q1;
            q3 = 4 * q3;
            inv = 1.0 / (q0 * q3 - q1 * q1);
        }
        if (CLK) __syncthreads();
        const unsigned long long c2 = CLK ? clock64() : 0;
        // the sums of one sweep from iterate buffer `in` (in < 0: x_0 = 0), solve_vals' solve
        auto sweep_r = [&](int in, double& r0, double& r1) {
            double s0 = 0.0, s1 = 0.0;
            // (one exposed LDS latency per edge; issuing all eight reads first and selecting the
            // missing diagonals away measured slower: the work of the missing edges and the
            // register pressure cost more than the latency)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (!(em & (1u << k))) continue;
                double gxj = 0.0, gyj = 0.0;
                if (in >= 0) {
                    const double2 gj = sg[in][nb[k]];
                    gxj = gj.x;
                    gyj = gj.y;
                }
                const double df2 = -ex[k] * gxj - ey[k] * gyj;
                const double w = c6[k] - 2 * df2;
                const double wx = ex[k] * r3[k], wy = ey[k] * r3[k];
                s0 = __builtin_fma(w, wx, s0);
                s1 = __builtin_fma(w, wy, s1);
            }
            r0 = (q3 * s0 - q1 * s1) * inv;
            r1 = (-q1 * s0 + q0 * s1) * inv;
        };
        for (int j = 1; j <= K; ++j) {
            if (dep >= j) {  // the square [j, W - 1 - j]^2 (depth >= j)
                const int in = j == 1 ? -1 : ((j - 1) & 1), out = j & 1;
                const ConeStep st = a.st[j];
                double r0, r1;
                sweep_r(in, r0, r1);
                double ox, oy;
                if (st.mode == 2) {
                    const double2 pv = sg[out][b];  // x_{j-2}, overwritten below
                    ox = st.omega * (-r0 - pv.x) + pv.x;
                    oy = st.omega * (-r1 - pv.y) + pv.y;
                } else if (st.mode == 1) {
                    ox = st.omega * (-r0 - 0.0) + 0.0;
                    oy = st.omega * (-r1 - 0.0) + 0.0;
                } else {
                    ox = -r0;
                    oy = -r1;
                }
                sg[out][b] = make_double2(ox, oy);
            }
            __syncthreads();  // (the first also waits for the next box's DMA: it had setup + sweep 1 to land)
        }
        const unsigned long long c3 = CLK ? clock64() : 0;
        // the cell's corners (the innermost ring): x_K out, and the change one more (plain-measured)
        // sweep would make
        if (dep == K + 1) {
            const int fin = K & 1;
            const double2 gk = sg[fin][b];
            const int64_t i = (int64_t)(R0 + r) * g.nh + (C0 + c);
            a.gout[2 * i] = gk.x;
            a.gout[2 * i + 1] = gk.y;
            if (a.chg) {
                double r0, r1;
                sweep_r(fin, r0, r1);
                const double cm = fmax(fabs(gk.x + r0), fabs(gk.y + r1)) / fmax(1.0, fmax(fabs(r0), fabs(r1)));
                cmax = fmax(cmax, cm);
            }
        }
        if (CLK && t == 0) {
            atomicAdd(a.clk, c1 - c0);
            atomicAdd(a.clk + 1, c2 - c1);
            atomicAdd(a.clk + 2, c3 - c2);
            atomicAdd(a.clk + 3, clock64() - c3);
            atomicAdd(a.clk + 4, 1ull);
        }
    }
    if (a.chg && dep == K + 1 && cmax > 0) atomicMax(a.chg, (unsigned long long)__double_as_longlong(cmax));
}

// vertex `idx` of the box in order of depth from the centre outwards (k_gd_cone_patch1's order):
// (r, c) and its depth d = min(r, c, W-1-r, W-1-c); indices [0, (W - 2j)^2) are the vertices of
// depth >= j. dep = 0 past the last (depth-1) vertex.
__device__ __forceinline__ void depth_order(int W, int idx, int& r, int& c, int& dep) {
    r = -1;
    c = -1;
    dep = 0;
    int rem = idx;
    for (int d = W / 2 - 1; d >= 1; --d) {
        const int s1 = W - 2 * d - 1, cnt = 4 * s1;
        if (rem < cnt) {
            if (rem < s1) { r = d; c = d + rem; }
            else if (rem < 2 * s1) { r = d + (rem - s1); c = d + s1; }
            else if (rem < 3 * s1) { r = d + s1; c = d + s1 - (rem - 2 * s1); }
            else { r = d + s1 - (rem - 3 * s1); c = d; }
            dep = d;
            return;
        }
        rem -= cnt;
    }
}

// k_gd_cone_patch1 as a two-stage pipeline over the workgroup's cells: threads [0, N1) hold the
// (W-2)^2 vertices of depth >= 1 of cell p and run its sweeps 1 .. S, while threads [N1, N1 + N2)
// hold the N2 = (W - 2S - 2)^2 vertices of depth >= S + 1 of cell p - 1 and run its sweeps
// S + 1 .. K and its corners' output - the late sweeps, a few waves each, no longer run alone.
// Each stage's threads compute their vertex's edge constants from that cell's box; box sets rotate
// over three (stage 1, stage 2, the next cell's DMA) and iterate buffer pairs over two (stage 2
// reads x_S, x_{S-1} where stage 1 left them). Per vertex the arithmetic is k_gd_cone_patch1's:
// the same bits. The host picks S (the smallest >= K/2 with N1 + N2 <= 1024).
template <bool CLK, bool RPF>
__global__ void __launch_bounds__(1024) k_gd_cone_patch2(Grid g, ConePatch<1> a, int S) {
    constexpr int P = 33;
    __shared__ double sxyf[3][3][P * 32];
    __shared__ double2 sg[2][2][P * 32];
    __shared__ uint8_t sd[3][P * 32];
    __shared__ int2 scell[1024];            // this workgroup's cells' box origins (R0, C0), read once
    __shared__ double sout[4][4];           // stage 2's corner results, stored one step later
    const int K = a.K, W = 2 * K + 4;
    const int t = threadIdx.x;
    const int N1 = (W - 2) * (W - 2), N2 = (W - 2 * S - 2) * (W - 2 * S - 2);
    const int role = t < N1 ? 1 : (t < N1 + N2 ? 2 : 0);
    int r, c, dep;
    depth_order(W, role == 1 ? t : t - N1, r, c, dep);
    if (role == 0) dep = 0;
    const int b = dep >= 1 ? r * P + c : 0;
    const int Q = max(S, K - S);
    const int count = *a.count;
    const int my = count > (int)blockIdx.x ? (count - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    const double* const gx_ = g.x;
    const double* const gy_ = g.y;
    const double* const gf_ = a.f;
    const uint8_t* const gd_ = g.diag;
    const int nh = g.nh;
    // the cell list into LDS first (the host keeps it <= 1024 cells per workgroup), so no wait on a
    // global load sits between a step's barrier and its DMA / setup
    for (int i = t; i < my; i += 1024) {
        const int64_t cell = a.cells[blockIdx.x + (int64_t)i * gridDim.x];
        const int iv0 = (int)(cell / (nh - 1)), ih0 = (int)(cell - (int64_t)iv0 * (nh - 1));
        scell[i] = make_int2(iv0 - (K + 1), ih0 - (K + 1));
    }
    __syncthreads();
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
    const int lr = t / 32, lc = t - (t / 32) * 32;
    // cell i's box: diagonal bytes into a register, x, y, f by DMA into box set st (k_gd_cone_patch1).
    // (The DMA issued at a step's start lands ~10k cycles after that step's sweeps have ended - its
    // LDS writes seem to queue behind the sweeps' traffic - yet it beats loading the next box
    // through registers on spare waves during the sweeps: 1.05 ms vs 0.47 ms, each global load's
    // latency then sits inside a sweep.)
    auto prefetch = [&](int i, int st, uint8_t& d) {
        const int2 o = scell[i];
        const int R0 = o.x, C0 = o.y;
        if (lr < W - 1 && lc < W - 1) d = gd_[(int64_t)(R0 + lr) * (nh - 1) + (C0 + lc)];
#pragma unroll
        for (int arr = 0; arr < 3; ++arr) {
            const double* base = arr == 0 ? gx_ : arr == 1 ? gy_ : gf_;
            for (int row = wv; row < W; row += 16) {
                const double* src = base + (int64_t)(R0 + row) * nh + C0;
                if (lane < 2 * W)
                    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) const char*)src + lane * 4,
                                                     (__attribute__((address_space(3))) void*)&sxyf[st][arr][row * P],
                                                     4, 0, 0);
            }
        }
    };
    uint8_t pd = 0;
    if (my > 0) prefetch(0, 0, pd);
    // the change measure's running max over this workgroup's cells (threads 0..3), one atomic at the
    // end: an atomicMax per cell on the one address queued at L2 behind every other workgroup's and
    // held each step's top (its vmcnt wait) for ~10k cycles
    double cmax = 0.0;
    for (int p = 0; p <= my; ++p) {
        const int s1 = p % 3, s2 = (p + 2) % 3;  // box sets of cell p (stage 1) and cell p - 1 (stage 2)
        const unsigned long long c0 = CLK ? clock64() : 0;
        if (p < my && lr < W && lc < W) sd[s1][lr * P + lc] = pd;
        if (!RPF || p == 0) __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA rows of cell p have landed
        const unsigned long long c0b = CLK ? clock64() : 0;
        if (RPF) {
            // cell p's box came through registers to LDS last step: an LDS-only barrier, so no wave
            // waits here for the acks of its earlier global stores (__syncthreads' fence would)
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        } else {
            __syncthreads();  // every wave's DMA has landed; the previous step's reads are done
        }
        const unsigned long long c1 = CLK ? clock64() : 0;
        double rx_ = 0.0, ry_ = 0.0, rf_ = 0.0;  // RPF: cell p + 1's box point through registers
        if (p + 1 < my) {
            pd = 0;
            if (RPF) {
                const int2 o = scell[p + 1];
                if (lr < W && lc < W) {
                    const int64_t q = (int64_t)(o.x + lr) * nh + (o.y + lc);
                    rx_ = gx_[q];
                    ry_ = gy_[q];
                    rf_ = gf_[q];
                    if (lr < W - 1 && lc < W - 1) pd = gd_[(int64_t)(o.x + lr) * (nh - 1) + (o.y + lc)];
                }
            } else {
                prefetch(p + 1, (p + 1) % 3, pd);
            }
        }
        if (p < my && lr < W && lc < W) sg[p & 1][0][lr * P + lc] = make_double2(0.0, 0.0);  // x_0
        if (p >= 2 && t >= 1020) {  // cell p - 2's corners, left by the last step's stage 2 (stored by
            const int q = t - 1020;    // the last wave: no box loads of its own for K <= 13)
            const int64_t i = (int64_t)sout[q][2];
            a.gout[2 * i] = sout[q][0];
            a.gout[2 * i + 1] = sout[q][1];
            cmax = fmax(cmax, sout[q][3]);
        }
        const bool act = dep >= 1 && (role == 1 ? p < my : p >= 1);
        const int bs = role == 1 ? s1 : s2;
        double2(*const gg)[P * 32] = sg[role == 1 ? (p & 1) : ((p + 1) & 1)];
        const double* const sx = sxyf[bs][0];
        const double* const sy = sxyf[bs][1];
        const double* const sf = sxyf[bs][2];
        const uint8_t* const sdd = sd[bs];
        int nb[8];
        unsigned em = 0;
        double ex[8], ey[8], r3[8], c6[8];
        double q0 = 0.0, q1 = 0.0, q3 = 0.0, inv = 0.0;
        if (act) {
            nb[0] = b - 1;
            nb[1] = b + 1;
            nb[2] = b - P;
            nb[3] = b + P;
            nb[4] = b - P - 1;
            nb[5] = b - P + 1;
            nb[6] = b + P - 1;
            nb[7] = b + P + 1;
            em = 0x0fu | (sdd[b - P - 1] == 0 ? 0x10u : 0u) | (sdd[b - P] == 1 ? 0x20u : 0u) |
                 (sdd[b - 1] == 1 ? 0x40u : 0u) | (sdd[b] == 0 ? 0x80u : 0u);
            const double xi = sx[b], yi = sy[b], fi = sf[b];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                ex[k] = ey[k] = r3[k] = c6[k] = 0.0;
                if (!(em & (1u << k))) continue;
                const int j = nb[k];
                const double exk = sx[j] - xi, eyk = sy[j] - yi;
                const double l2 = exk * exk + eyk * eyk;
                double rr = __builtin_amdgcn_rsq(l2);
                rr = rr * __builtin_fma(-0.5 * l2 * rr, rr, 1.5);
                const double r3k = rr * rr * rr;
                const double wx = exk * r3k, wy = eyk * r3k;
                q0 = __builtin_fma(exk, wx, q0);
                q1 = __builtin_fma(exk, wy, q1);
                q3 = __builtin_fma(eyk, wy, q3);
                ex[k] = exk;
                ey[k] = eyk;
                r3[k] = r3k;
                c6[k] = 6 * (fi - sf[j]);
            }
            q0 = 4 * q0;
            q1 = 4 * q1;
            q3 = 4 * q3;
            inv = 1.0 / (q0 * q3 - q1 * q1);
        }
        if (RPF && p + 1 < my && lr < W && lc < W) {  // after setup: its latency was the setup's time
            const int q = lr * P + lc, st = (p + 1) % 3;
            sxyf[st][0][q] = rx_;
            sxyf[st][1][q] = ry_;
            sxyf[st][2][q] = rf_;
        }
        // x_0 in place for sweep 1 (LDS only: the next box's DMA stays in flight)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const unsigned long long c2 = CLK ? clock64() : 0;
        // the sums of one sweep from iterate buffer `in` (sweep 1 reads x_0 = 0 from buffer 0, zeroed
        // at the step's top), solve_vals' solve; the buffer's row base is formed once per sweep, so
        // each edge's read is one LDS instruction with a constant offset
        auto sweep_r = [&](int in, double& r0, double& r1) {
            constexpr int off[8] = {-1, 1, -P, P, -P - 1, -P + 1, P - 1, P + 1};
            double s0 = 0.0, s1 = 0.0;
            const double2* const gi = gg[in] + b;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (!(em & (1u << k))) continue;
                const double2 gj = gi[off[k]];
                const double df2 = -ex[k] * gj.x - ey[k] * gj.y;
                const double w = c6[k] - 2 * df2;
                const double wx = ex[k] * r3[k], wy = ey[k] * r3[k];
                s0 = __builtin_fma(w, wx, s0);
                s1 = __builtin_fma(w, wy, s1);
            }
            r0 = (q3 * s0 - q1 * s1) * inv;
            r1 = (-q1 * s0 + q0 * s1) * inv;
        };
        for (int q = 1; q <= Q; ++q) {
            const int j = role == 1 ? q : S + q;
            if (act && dep >= j && (role == 1 ? q <= S : j <= K)) {
                const int in = (j - 1) & 1, out = j & 1;
                const ConeStep st = a.st[j];
                double r0, r1;
                sweep_r(in, r0, r1);
                double ox, oy;
                if (st.mode == 2) {
                    const double2 pv = gg[out][b];  // x_{j-2}, overwritten below
                    ox = st.omega * (-r0 - pv.x) + pv.x;
                    oy = st.omega * (-r1 - pv.y) + pv.y;
                } else if (st.mode == 1) {
                    ox = st.omega * (-r0 - 0.0) + 0.0;
                    oy = st.omega * (-r1 - 0.0) + 0.0;
                } else {
                    ox = -r0;
                    oy = -r1;
                }
                gg[out][b] = make_double2(ox, oy);
            }
            // LDS-only barrier: __syncthreads' fence would also wait (vmcnt) for the next box's DMA
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
        const unsigned long long c3 = CLK ? clock64() : 0;
        // cell p - 1's corners (stage 2's innermost ring): x_K and the change of one more sweep, into
        // LDS; threads 0..3 store them after the next step's barrier (or below, after the last step),
        // so the stores' latency is not waited for at the next step's top
        if (role == 2 && act && dep == K + 1) {
            const int2 o = scell[p - 1];
            const int fin = K & 1;
            const double2 gk = gg[fin][b];
            double cm = 0.0;
            if (a.chg) {
                double r0, r1;
                sweep_r(fin, r0, r1);
                cm = fmax(fabs(gk.x + r0), fabs(gk.y + r1)) / fmax(1.0, fmax(fabs(r0), fabs(r1)));
            }
            const int q = t - N1;  // the innermost ring: stage 2's first four threads
            sout[q][0] = gk.x;
            sout[q][1] = gk.y;
            sout[q][2] = (double)((int64_t)(o.x + r) * nh + (o.y + c));
            sout[q][3] = cm;
        }
        if (p == my && my >= 1) {  // the last cell's corners
            __syncthreads();
            if (t >= 1020) {
                const int q = t - 1020;
                const int64_t i = (int64_t)sout[q][2];
                a.gout[2 * i] = sout[q][0];
                a.gout[2 * i + 1] = sout[q][1];
                cmax = fmax(cmax, sout[q][3]);
            }
        }
        if (CLK && t == 0) {
            atomicAdd(a.clk, c1 - c0);
            atomicAdd(a.clk + 1, c2 - c1);
            atomicAdd(a.clk + 2, c3 - c2);
            atomicAdd(a.clk + 3, clock64() - c3);
            atomicAdd(a.clk + 4, 1ull);
            atomicAdd(a.clk + 5, c0b - c0);
        }
    }
    if (a.chg && t >= 1020 && cmax > 0) atomicMax(a.chg, (unsigned long long)__double_as_longlong(cmax));
}

// targets -> interior target cells (the patch list) and whether any target needs the band
__global__ void __launch_bounds__(kBlock) k_gd_cone_targets(Grid g, const int* __restrict__ owner, int64_t m, int K,
                                                             int64_t* cells, int* count, int* band) {
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
__global__ void __launch_bounds__(kAxesThreads) k_gd_axes(const double* __restrict__ rx, const double* __restrict__ ry,
                                                          int64_t L, int mx, int my, double* gx, double* gy,
                                                          double* ext) {
    __shared__ double red[4][kAxesThreads / 64];
    double lo_x = INFINITY, hi_x = -INFINITY, lo_y = INFINITY, hi_y = -INFINITY;
    for (int64_t r = threadIdx.x; r < L; r += blockDim.x) {
        lo_x = fmin(lo_x, rx[r]);
        hi_x = fmax(hi_x, rx[r]);
        lo_y = fmin(lo_y, ry[r]);
        hi_y = fmax(hi_y, ry[r]);
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
    auto lin = [&](double a0, double a1, int m, double* out) {
        if (m == 1) {
            if (threadIdx.x == 0) out[0] = a0;
            return;
        }
        const double step = (a1 - a0) / (double)(m - 1);
        for (int i = threadIdx.x; i < m; i += blockDim.x) {
            double v;
            if (step == 0) v = (double)i / (double)(m - 1) * (a1 - a0) + a0;  // numpy's zero-step branch
            else v = (double)i * step + a0;
            out[i] = i == m - 1 ? a1 : v;
        }
    };
    lin(e[0], e[1], mx, gx);
    lin(e[2], e[3], my, gy);
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
        const double* a = w == 0 ? gx : gy;
        const int m = w == 0 ? mx : my;
        double sum;
        if (w == 0) sum = pw_sum_wave_get(tree[0], [=](int i) { return gx[i % mx]; }, cnt);
        else sum = pw_sum_wave_get(tree[1], [=](int i) { return gy[i / mx]; }, cnt);
        const double mean = sum / (double)cnt;
        if ((threadIdx.x & 63) == 0) ext[4 + w] = m > 1 ? fabs((a[1] - mean) - (a[0] - mean)) : 0.0;
    }
}

// a sharded lattice's targets: this rank forms the interior targets whose cell's p00 lies in its
// rays [own0, own1); the band owner forms every band and pocket target. assigned[t] = 1 for the
// targets formed here; the interior ones' cells go to the patch list
__global__ void __launch_bounds__(kBlock) k_gd_cone_assign(Grid g, const int* __restrict__ owner, int64_t m, int K,
                                                            int64_t own0, int64_t own1, int band_on, int64_t* cells,
                                                            int* count, int* band, uint8_t* assigned) {
    const int64_t nc2 = 2 * ncells(g);
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < m; t += (int64_t)gridDim.x * blockDim.x) {
        const int o = owner[t];
        uint8_t mine = 0;
        if (o != INT32_MAX) {
            bool interior = false;
            int64_t c = -1, p00 = -1;
            if (o < nc2) {
                c = o >> 1;
                const int iv = (int)(c / (g.nh - 1)), ih = (int)(c - (int64_t)iv * (g.nh - 1));
                interior = iv - K - 1 >= 1 && iv + K + 2 <= g.nv - 2 && ih - K - 1 >= 1 && ih + K + 2 <= g.nh - 2;
                p00 = (int64_t)iv * g.nh + ih;
            }
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

// ------------------------------------------------------------------ targets

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

// cell triangles (ids < 2 * ncells): one thread each, a box of a few targets
__global__ void __launch_bounds__(kBlock) k_gd_claim(Grid g, Targets t, int* owner) {
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
// held to each triangle's exact box and barycentric test, so the claims are k_gd_claim's
// candidate index range of the targets of an ascending linspace axis a (m points) in [lo, hi):
// the real-valued indices of lo and hi from the axis's own step, widened by 1e-6 of an index (the
// axis values sit within a few ulp of a0 + c * step); empty when no integer falls between them
__device__ __forceinline__ bool axis_range(const double* a, int m, double inv_step, double lo, double hi, int& c0,
                                           int& c1) {
    const double a0 = a[0];
    const double e0 = (lo - a0) * inv_step - 1e-6, e1 = (hi - a0) * inv_step + 1e-6;
    if (!(e1 >= 0.0) || !(e0 <= (double)(m - 1))) return false;
    const double f0 = ceil(fmax(e0, 0.0)), f1 = floor(fmin(e1, (double)(m - 1)));
    if (f0 > f1) return false;
    c0 = (int)f0;
    c1 = (int)f1 + 1;
    return true;
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

// one cell's claims (its two triangles' targets)
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

// the claim kernels' axis test: whether both axes are linspaces (workgroup-wide; every thread)
__device__ __forceinline__ bool axes_uniform(const Targets& t) {
    // the index-box estimate needs evenly spaced axes (np.linspace, the driver's); any other
    // ascending axis takes the exact binary search (lower_idx) of the per-triangle claim
    bool ok = true;
    for (int i = threadIdx.x; i < t.mx || i < t.my; i += blockDim.x)
        ok = ok && axis_uniform_part(t.gx, t.mx, i) && axis_uniform_part(t.gy, t.my, i);
    return __syncthreads_and(ok) != 0;
}

__global__ void __launch_bounds__(kBlock) k_gd_claim_cells(Grid g, Targets t, int* owner) {
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
// threads idle on the common few-target boxes)
__global__ void __launch_bounds__(kBlock) k_gd_claim_pockets(Grid g, Targets t, int* owner) {
    const int64_t nc2 = 2 * ncells(g);
    const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
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

__device__ double clough_tocher(const Grid& g, int64_t tid, const Tri& T, const double* f, const double* grad,
                                const double (&b)[3]) {
    const double p0x = g.x[T.v[0]], p0y = g.y[T.v[0]];
    const double p1x = g.x[T.v[1]], p1y = g.y[T.v[1]];
    const double p2x = g.x[T.v[2]], p2y = g.y[T.v[2]];
    const double e12x = p1x - p0x, e12y = p1y - p0y;
    const double e23x = p2x - p1x, e23y = p2y - p1y;
    const double e31x = p0x - p2x, e31y = p0y - p2y;
    const double f1 = f[T.v[0]], f2 = f[T.v[1]], f3 = f[T.v[2]];
    const double g0x = grad[2 * T.v[0]], g0y = grad[2 * T.v[0] + 1];
    const double g1x = grad[2 * T.v[1]], g1y = grad[2 * T.v[1] + 1];
    const double g2x = grad[2 * T.v[2]], g2y = grad[2 * T.v[2] + 1];
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
        const int64_t n = tri_nbr(g, tid, k);
        if (n < 0) {
            gk[k] = -0.5;
            continue;
        }
        const Tri N = tri_verts(g, n);
        const double cx = (g.x[N.v[0]] + g.x[N.v[1]] + g.x[N.v[2]]) / 3;
        const double cy = (g.y[N.v[0]] + g.y[N.v[1]] + g.y[N.v[2]]) / 3;
        double c[3];
        bary(g, T, cx, cy, c);
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

// nvals value sets share the triangulation: f / grad / out strided by n / 2n / mx*my
__global__ void __launch_bounds__(kBlock) k_gd_eval(Grid g, Targets t, const int* __restrict__ owner,
                                                    const double* f, const double* grad, int nvals, double* out) {
    const int64_t m = (int64_t)t.mx * t.my, n = (int64_t)g.nv * g.nh;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const int o = owner[i];
        if (o == INT32_MAX) {
            for (int v = 0; v < nvals; ++v) out[v * m + i] = __builtin_nan("");
            continue;
        }
        const int r = (int)(i / t.mx), c = (int)(i - (int64_t)r * t.mx);
        const Tri T = tri_verts(g, o);
        double b[3];
        bary(g, T, t.gx[c], t.gy[r], b);
        for (int v = 0; v < nvals; ++v) out[v * m + i] = clough_tocher(g, o, T, f + v * n, grad + 2 * v * n, b);
    }
}

// k_gd_eval for the targets a rank forms (assigned): value and count, zeros elsewhere, so the
// ranks' pieces add up to the map (a SUM reduction; count 0: outside the hull, NaN)
__global__ void __launch_bounds__(kBlock) k_gd_eval_part(Grid g, Targets t, const int* __restrict__ owner,
                                                         const uint8_t* __restrict__ assigned, const double* f,
                                                         const double* grad, int nvals, double* out, double* cnt) {
    const int64_t m = (int64_t)t.mx * t.my, n = (int64_t)g.nv * g.nh;
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
    }
}

// the assembled pieces: value where some rank formed it, NaN elsewhere (outside the hull)
__global__ void k_gd_part_finish(double* out, const double* cnt, int64_t m, int nvals) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        if (!(cnt[i] > 0))
            for (int v = 0; v < nvals; ++v) out[v * m + i] = __builtin_nan("");
}

__global__ void k_fill_i32(int* p, int64_t n, int v) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

// A/B knobs (environment, read once): workgroup cap of the sweep / claim launches, and the
// per-sweep change reduction switched off (timing only)
int64_t gd_grid_cap() {
    static int64_t g = [] {
        const char* e = getenv("AKB_GD_GRID");
        const long long v = e ? atoll(e) : 0;
        return (int64_t)(v >= 64 ? v : kStreamGridCap);
    }();
    return g;
}
int gd_no_xcd() {
    static int b = getenv("AKB_GD_NOXCD") != nullptr ? 1 : 0;
    return b;
}
bool gd_claim_v1() {  // A/B: the per-cell claim kernel
    static bool b = getenv("AKB_GD_CLAIM_V1") != nullptr;
    return b;
}
bool gd_cells_v1() {  // A/B: the per-cell (untiled) cell pass
    static bool b = getenv("AKB_GD_CELLS_V1") != nullptr;
    return b;
}
// the cell pass over the window's `rows` cell rows
int launch_cells(const Grid& g, uint8_t* diag, double tol, unsigned* d_flags, int rows, hipStream_t s) {
    const int64_t wc = (int64_t)rows * (g.nh - 1);
    if (gd_cells_v1()) {
        k_gd_cells<<<grid_for(wc, 1, kStreamGridCap), kBlock, 0, s>>>(g, diag, tol, d_flags);
    } else {
        const int64_t tiles = (int64_t)((rows + kCellTile - 1) / kCellTile) * ((g.nh - 1 + kCellTile - 1) / kCellTile);
        k_gd_cells_tiled<<<(unsigned)(tiles < 4096 ? tiles : 4096), kCellTile * kCellTile, 0, s>>>(g, diag, tol,
                                                                                                    d_flags);
    }
    return launch_status("k_gd_cells");
}
bool gd_band_split() {  // the band sweep as two launches (band, then ring); AKB_GD_BAND_MERGED: one
    // with a wave per ring vertex (measured slower: 37 us vs 16 + 13 per sweep beside the passes -
    // the ring's grid edges then wait behind its chord reduction on one lane)
    static bool b = getenv("AKB_GD_BAND_MERGED") == nullptr;
    return b;
}
bool gd_band_sweep8() {  // one launch per band sweep, the ring in 8-lane groups (A/B: AKB_GD_BAND_SPLIT)
    static bool b = getenv("AKB_GD_BAND_SPLIT") == nullptr && getenv("AKB_GD_BAND_MERGED") == nullptr;
    return b;
}
bool gd_patch_rowmajor() {  // A/B: the register patch kernel's lanes along rows (not by depth)
    static bool b = getenv("AKB_GD_PATCH_ROWMAJOR") != nullptr;
    return b;
}
bool gd_patch_rpf() {  // the pipeline's next box through registers over the setup (A/B: AKB_GD_PATCH_DMA,
    // the LDS DMA issued at the step's top: 433-444 vs 423-426 us, same bits)
    static bool b = getenv("AKB_GD_PATCH_DMA") == nullptr;
    return b;
}
bool gd_patch_pipe() {  // the two-stage patch pipeline (A/B: AKB_GD_PATCH_NOPIPE)
    static bool b = getenv("AKB_GD_PATCH_NOPIPE") == nullptr;
    return b;
}
bool gd_patch_prefetch() {  // the next cell's box fetched into registers during the sweeps (A/B: off)
    static bool b = getenv("AKB_GD_PATCH_NOPREFETCH") == nullptr;
    return b;
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
unsigned long long* gd_patch_clock() {  // diagnostics: per-phase cycle sums of the register patch kernel
    static unsigned long long* p = [] {
        unsigned long long* q = nullptr;
        if (getenv("AKB_GD_PATCH_CLOCK") && hipMalloc(&q, 8 * sizeof(unsigned long long)) != hipSuccess) q = nullptr;
        return q;
    }();
    return p;
}
bool gd_patch_v1() {  // A/B: the 256-thread patch kernel for one value set
    static bool b = getenv("AKB_GD_PATCH_V1") != nullptr;
    return b;
}
bool gd_no_change() {
    static bool b = getenv("AKB_GD_NOCHG") != nullptr;
    return b;
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

// one Jacobi sweep; d_change: largest relative change (as ordered double bits, zeroed by the
// caller); nvals value sets strided by n (values) and 2n (gradients); ring_work: 10 L doubles.
// gprev != NULL: Chebyshev step, gout = omega * (jacobi(gin) - gprev) + gprev (a Jacobi sweep
// then, whatever AKB_GD_GS says); gprev == NULL with omega == 0: a plain Jacobi sweep
int akb_gd_grad_sweep_f64(const double* x, const double* y, int nv, int nh, const uint8_t* diag, int npock,
                          const int32_t* ptri, const int32_t* pnbr, const int32_t* edge_tri, const int32_t* xptr,
                          const int32_t* xidx, const double* f, int nvals, const double* gin, const double* gprev,
                          double omega, double* gout, double* ring_work, unsigned long long* d_change, void* stream) {
    clear_error();
    AKB_REQUIRE(x && y && diag && f && gin && gout && ring_work && d_change && nvals >= 1, "bad arguments");
    AKB_REQUIRE(!gprev || (omega > 0 && omega < 2), "Chebyshev weight outside (0, 2)");
    Grid g{x, y, nv, nh, diag, npock, ptri, pnbr, edge_tri, xptr, xidx, gd_no_xcd()};
    {
        const char* re = getenv("AKB_GD_ROWS");
        const int rows = re ? atoi(re) : 0;
        if (rows >= 4 && rows <= 256) g.strip_rows = rows;
    }
    hipStream_t s = (hipStream_t)stream;
    const int64_t n = (int64_t)nv * nh;
    const int64_t L = 2 * (int64_t)(nh - 1) + 2 * (int64_t)(nv - 1);
    unsigned long long* chg = gd_no_change() ? nullptr : d_change;
    const int64_t chunks = (n + kGradChunk - 1) / kGradChunk;
    const unsigned gr = (unsigned)(8 * ((chunks + 7) / 8));  // a multiple of 8 for the XCD mapping
    const unsigned grr = grid_for(L * 64);
    // the LDS strip kernel, AKB_GD_STRIP columns wide (64 / 128 / 256; 0: the gather kernel; read
    // per call: the tests compare them)
    const char* se = getenv("AKB_GD_STRIP");
    // 256 by default: 11.9 vs 12.5 / 12.8 ms of sweeps for 128 / 64 on the C3 hits (the row chunk,
    // 8 ... 64 rows, moves it by < 5 %: the strips are LDS-occupancy bound at 3 waves per SIMD)
    int strip = se ? atoi(se) : 256;
    if (strip != 0 && strip != 64 && strip != 128 && strip != 256) strip = 256;
    // the strip sweeps as line Gauss-Seidel (AKB_GD_GS=0: Jacobi, the gather kernel's bits)
    const char* ge = getenv("AKB_GD_GS");
    // Gauss-Seidel only for a plain sweep that asks for it (omega >= 1): Chebyshev iterations pass
    // omega = 0 for their plain first sweep, which must be the Jacobi one
    const bool gs_sweep = !(ge && ge[0] == '0') && !gprev && omega > 0;
    const unsigned gs =
        strip ? (unsigned)(((nh + strip - 1) / strip) * ((nv + g.strip_rows - 1) / g.strip_rows)) : 0u;
    for (int v = 0; v < nvals; v += 2) {
        const double* fv = f + v * n;
        const double* gi = gin + 2 * v * n;
        double* go = gout + 2 * v * n;
        const Cheb ch{gprev ? gprev + 2 * v * n : nullptr, omega};
        if (nvals - v >= 2) {
            if (strip == 64)
                gs_sweep ? k_gd_grad_strip<2, 64, true><<<gs, 64, 0, s>>>(g, fv, gi, go, ring_work, chg, ch)
                         : k_gd_grad_strip<2, 64><<<gs, 64, 0, s>>>(g, fv, gi, go, ring_work, chg, ch);
            else if (strip == 128)
                gs_sweep ? k_gd_grad_strip<2, 128, true><<<gs, 128, 0, s>>>(g, fv, gi, go, ring_work, chg, ch)
                         : k_gd_grad_strip<2, 128><<<gs, 128, 0, s>>>(g, fv, gi, go, ring_work, chg, ch);
            else if (strip == 256)
                gs_sweep ? k_gd_grad_strip<2, 256, true><<<gs, 256, 0, s>>>(g, fv, gi, go, ring_work, chg, ch)
                         : k_gd_grad_strip<2, 256><<<gs, 256, 0, s>>>(g, fv, gi, go, ring_work, chg, ch);
            else
                k_gd_grad<2><<<gr, kBlock, 0, s>>>(g, fv, gi, go, ring_work, chg, ch);
            k_gd_grad_ring<2><<<grr, kBlock, 0, s>>>(g, fv, gi, go, ring_work, chg, ch);
        } else {
            if (strip == 64)
                gs_sweep ? k_gd_grad_strip<1, 64, true><<<gs, 64, 0, s>>>(g, fv, gi, go, ring_work, chg, ch)
                         : k_gd_grad_strip<1, 64><<<gs, 64, 0, s>>>(g, fv, gi, go, ring_work, chg, ch);
            else if (strip == 128)
                gs_sweep ? k_gd_grad_strip<1, 128, true><<<gs, 128, 0, s>>>(g, fv, gi, go, ring_work, chg, ch)
                         : k_gd_grad_strip<1, 128><<<gs, 128, 0, s>>>(g, fv, gi, go, ring_work, chg, ch);
            else if (strip == 256)
                gs_sweep ? k_gd_grad_strip<1, 256, true><<<gs, 256, 0, s>>>(g, fv, gi, go, ring_work, chg, ch)
                         : k_gd_grad_strip<1, 256><<<gs, 256, 0, s>>>(g, fv, gi, go, ring_work, chg, ch);
            else
                k_gd_grad<1><<<gr, kBlock, 0, s>>>(g, fv, gi, go, ring_work, chg, ch);
            k_gd_grad_ring<1><<<grr, kBlock, 0, s>>>(g, fv, gi, go, ring_work, chg, ch);
        }
        int st = launch_status("k_gd_grad");
        if (st) return st;
    }
    return 0;
}

// kk = 1 or 2 Jacobi sweeps in one launch of the register kernel, each a Chebyshev step (om1, om2;
// gprev == NULL: the first is a plain sweep; gin == NULL: x_k = 0). gout1 = x_{k+1}, gout2 =
// x_{k+2}; d_change[0], [1]: the sweeps' largest relative changes; ring_work: 14 L doubles.
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
    Grid g{x, y, nv, nh, diag, npock, ptri, pnbr, edge_tri, xptr, xidx, gd_no_xcd()};
    int rows = 24;  // rows per wave (AKB_GD_ROWS): 24 at 3 waves per SIMD measured best on the C3 hits
    {
        const char* re = getenv("AKB_GD_ROWS");
        const int v = re ? atoi(re) : 0;
        if (v >= 4 && v <= 1024) rows = v;
    }
    // the two-value two-sweep kernel's occupancy variant (AKB_GD_OCC, A/B): 3 waves per SIMD by
    // default (168 VGPRs, 12 B of scratch: 4.75 vs 5.3 ms for the C3 hits' solve at 2 waves)
    const char* oe = getenv("AKB_GD_OCC");
    const int occ = oe ? atoi(oe) : 3;
    hipStream_t s = (hipStream_t)stream;
    const int64_t n = (int64_t)nv * nh;
    const int64_t L = 2 * (int64_t)(nh - 1) + 2 * (int64_t)(nv - 1);
    unsigned long long* chg = gd_no_change() ? nullptr : d_change;
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
        double* acc = ring_work + 7 * L;
        if (nv2 == 2) {
            k_gd_ring_chords<2><<<grr, kBlock, 0, s>>>(g, fv, gi, chords);
            SweepArgs<2> a{fv, gi, gprev ? gprev + 2 * v * n : nullptr, om1, om2, o1, o2, chords, acc, chg, rows};
            if (kk == 2 && occ == 2) k_gd_sweeps<2, 2, 1, 2><<<gw, 256, 0, s>>>(g, a);
            else if (kk == 2 && occ == 5) k_gd_sweeps<2, 2, 3, 2><<<gw, 256, 0, s>>>(g, a);
            else if (kk == 2 && occ == 3) k_gd_sweeps<2, 2, 3><<<gw, 256, 0, s>>>(g, a);
            else if (kk == 2 && occ == 4) k_gd_sweeps<2, 2, 4><<<gw, 256, 0, s>>>(g, a);
            else if (kk == 2) k_gd_sweeps<2, 2, 1><<<gw, 256, 0, s>>>(g, a);
            else k_gd_sweeps<2, 1, 1><<<gw, 256, 0, s>>>(g, a);
            if (kk == 2)
                k_gd_grad_ring<2><<<grr, kBlock, 0, s>>>(g, fv, o1, o2, acc, chg ? chg + 1 : nullptr,
                                                         Cheb{gi, om2, gi ? 0 : 1});
        } else {
            k_gd_ring_chords<1><<<grr, kBlock, 0, s>>>(g, fv, gi, chords);
            SweepArgs<1> a{fv, gi, gprev ? gprev + 2 * v * n : nullptr, om1, om2, o1, o2, chords, acc, chg, rows};
            if (kk == 2) k_gd_sweeps<1, 2, 1><<<gw, 256, 0, s>>>(g, a);
            else k_gd_sweeps<1, 1, 1><<<gw, 256, 0, s>>>(g, a);
            if (kk == 2)
                k_gd_grad_ring<1><<<grr, kBlock, 0, s>>>(g, fv, o1, o2, acc, chg ? chg + 1 : nullptr,
                                                         Cheb{gi, om2, gi ? 0 : 1});
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
    if (getenv("AKB_GD_CLAIM_TRI"))  // the per-triangle claim (A/B and the tests' cross-check)
        k_gd_claim<<<grid_for(ntri - npock, 1, gd_grid_cap()), kBlock, 0, s>>>(g, t, owner);
    else if (gd_claim_v1())
        k_gd_claim_cells<<<grid_for((ntri - npock) / 2, 1, kStreamGridCap), kBlock, 0, s>>>(g, t, owner);
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
    return (3 * (int64_t)nv2 * n * 2 * 8 + L * 7 * 8 + m * 8 + m + 64 + 63) / 64 * 64;
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
        if (gd_claim_v1()) {
            k_gd_claim_cells<<<grid_for(wc, 1, kStreamGridCap), kBlock, 0, s>>>(g, t, owner);
        } else if (scratch) {
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
// as k_gd_eval_part writes them (cnt == nullptr: k_gd_eval's NaN for unclaimed targets)
int cone_part(const Grid& g, const Targets& t, int64_t own0, int64_t own1, int band_on, const double* f, int nvals,
              int K, const double* omegas, void* work, const int* owner, double* out, double* cnt,
              unsigned long long* d_change, hipStream_t s) {
    const int64_t n = (int64_t)g.nv * g.nh, m = (int64_t)t.mx * t.my;
    const int64_t L = 2 * (int64_t)(g.nh - 1) + 2 * (int64_t)(g.nv - 1);
    const int nv2 = nvals >= 2 ? 2 : 1;
    double* gb[3];
    for (int k = 0; k < 3; ++k) gb[k] = (double*)work + (int64_t)k * nv2 * n * 2;
    double* ring_acc = (double*)work + 3 * (int64_t)nv2 * n * 2;
    int64_t* cells = (int64_t*)(ring_acc + L * 7);
    uint8_t* assigned = (uint8_t*)(cells + m);
    int* count = (int*)(((uintptr_t)(assigned + m) + 7) & ~(uintptr_t)7);
    int* band = count + 1;
    if (hipMemsetAsync(count, 0, 2 * sizeof(int), s) != hipSuccess) return launch_status("hipMemsetAsync");
    k_gd_cone_assign<<<grid_for(m, 1), kBlock, 0, s>>>(g, owner, m, K, own0, own1, band_on, cells, count, band,
                                                      assigned);
    int st = launch_status("k_gd_cone_assign");
    if (st) return st;
    // the boundary band, shrinking like the patches' squares: sweep j forms depth <= 2K + 3 - j, whose
    // neighbours (depth <= 2K + 4 - j) sweep j - 1 formed, so x_K is the global iteration's to depth
    // K + 3 >= every band target's corners (the first sweep reads x_0 = 0 only)
    ConeStep steps[kConeMaxK + 1];
    steps[0] = ConeStep{0, 1.0};
    for (int j = 1; j <= K; ++j)
        steps[j] = j == 1 ? ConeStep{0, 1.0} : j == 2 ? ConeStep{1, omegas[1]} : ConeStep{2, omegas[j - 1]};
    const unsigned pg = (unsigned)(m < 8192 ? m : 8192);
    for (int v0 = 0; v0 < nvals; v0 += 2) {
        const int nvv = nvals - v0 >= 2 ? 2 : 1;
        const double* fv = f + v0 * n;
        if (band_on) {
            for (int j = 1; j <= K; ++j) {
                const double* gin = j == 1 ? nullptr : gb[(j - 1) % 3];
                const double* gprev = j >= 3 ? gb[(j + 1) % 3] : nullptr;
                const BandMap bm = band_map(g.nv, g.nh, 2 * K + 3 - j);
                const unsigned nbw = grid_for(bm.total, 1, kStreamGridCap), nrw = grid_for(L * 64), nr8 = grid_for((L + 7) / 8 * 64);
                if (nvv == 2) {
                    ConeBand<2> a{fv, gin, gprev, gb[j % 3], ring_acc, steps[j], band};
                    if (gd_band_sweep8()) {
                        k_gd_cone_sweep8<2><<<nbw + nr8, kBlock, 0, s>>>(g, bm, a, (int)nbw);
                    } else if (gd_band_split()) {
                        k_gd_cone_band<2><<<nbw, kBlock, 0, s>>>(g, bm, a);
                        k_gd_cone_ring<2><<<nr8, kBlock, 0, s>>>(g, a);
                    } else {
                        k_gd_cone_sweep<2><<<nbw + nrw, kBlock, 0, s>>>(g, bm, a, (int)nbw);
                    }
                } else {
                    ConeBand<1> a{fv, gin, gprev, gb[j % 3], ring_acc, steps[j], band};
                    if (gd_band_sweep8()) {
                        k_gd_cone_sweep8<1><<<nbw + nr8, kBlock, 0, s>>>(g, bm, a, (int)nbw);
                    } else if (gd_band_split()) {
                        k_gd_cone_band<1><<<nbw, kBlock, 0, s>>>(g, bm, a);
                        k_gd_cone_ring<1><<<nr8, kBlock, 0, s>>>(g, a);
                    } else {
                        k_gd_cone_sweep<1><<<nbw + nrw, kBlock, 0, s>>>(g, bm, a, (int)nbw);
                    }
                }
                if ((st = launch_status("k_gd_cone_band"))) return st;
            }
        }
        if (nvv == 2) {
            ConePatch<2> a{fv, cells, count, K, {}, gb[K % 3], d_change};
            for (int j = 0; j <= K; ++j) a.st[j] = steps[j];
            k_gd_cone_patch<2><<<pg, 256, 0, s>>>(g, a);
        } else {
            ConePatch<1> a{fv, cells, count, K, {}, gb[K % 3], d_change};
            for (int j = 0; j <= K; ++j) a.st[j] = steps[j];
            if (gd_patch_v1())
                k_gd_cone_patch<1><<<pg, 256, 0, s>>>(g, a);
            else
            {
                unsigned long long* clk = gd_patch_clock();
                if (clk) {
                    (void)hipMemsetAsync(clk, 0, 8 * sizeof(unsigned long long), s);
                    a.clk = clk;
                }
                const int rm = gd_patch_rowmajor() ? 1 : 0;
                // the two-stage pipeline when both stages' vertices fit 1024 threads (K <= 14: always)
                int S = -1;
                if (gd_patch_pipe() && !rm) {
                    const int W = 2 * K + 4;
                    const char* es = getenv("AKB_GD_PATCH_S");  // A/B: the first sweep stage 2 does is S + 1
                    for (int s2 = es ? std::max(1, std::min(K, atoi(es))) : (K + 1) / 2; s2 <= K && S < 0; ++s2)
                        if ((W - 2) * (W - 2) + (W - 2 * s2 - 2) * (W - 2 * s2 - 2) <= 1024) S = s2;
                }
                // prefetching: one persistent workgroup per CU walks its cells (the next one's box
                // loads during the current one's sweeps); else workgroups per cell
                // A/B: AKB_GD_PATCH_GRID leaves CUs to the other streams' kernels while the patches run
                const char* eg = getenv("AKB_GD_PATCH_GRID");
                const unsigned pp = std::min(pg, eg ? std::max(1u, (unsigned)atoi(eg)) : gd_cu_count());
                if (S >= 0 && (int64_t)m > 1024 * (int64_t)pp) S = -1;  // the cell list fits LDS
                if (S >= 0) {
                    if (clk) {
                        if (gd_patch_rpf()) k_gd_cone_patch2<true, true><<<pp, 1024, 0, s>>>(g, a, S);
                        else k_gd_cone_patch2<true, false><<<pp, 1024, 0, s>>>(g, a, S);
                    } else {
                        if (gd_patch_rpf()) k_gd_cone_patch2<false, true><<<pp, 1024, 0, s>>>(g, a, S);
                        else k_gd_cone_patch2<false, false><<<pp, 1024, 0, s>>>(g, a, S);
                    }
                } else if (clk) {
                    if (gd_patch_prefetch()) k_gd_cone_patch1<true, true><<<pp, 1024, 0, s>>>(g, a, rm);
                    else k_gd_cone_patch1<false, true><<<pg, 1024, 0, s>>>(g, a, rm);
                } else {
                    if (gd_patch_prefetch()) k_gd_cone_patch1<true, false><<<pp, 1024, 0, s>>>(g, a, rm);
                    else k_gd_cone_patch1<false, false><<<pg, 1024, 0, s>>>(g, a, rm);
                }
                if (clk) {
                    unsigned long long h[8];
                    (void)hipMemcpyAsync(h, clk, sizeof(h), hipMemcpyDeviceToHost, s);
                    (void)hipStreamSynchronize(s);
                    const double nc = h[4] ? (double)h[4] : 1.0;
                    fprintf(stderr,
                            "AKB_GD_PATCH_CLOCK cells %llu cycles/cell: load %.0f (own vmem wait %.0f) setup %.0f sweeps "
                            "%.0f out %.0f\n",
                            h[4], h[0] / nc, h[5] / nc, h[1] / nc, h[2] / nc, h[3] / nc);
                }
            }
        }
        if ((st = launch_status("k_gd_cone_patch"))) return st;
        if (cnt)
            k_gd_eval_part<<<grid_for(m, 1, kStreamGridCap), kBlock, 0, s>>>(g, t, owner, assigned, fv, gb[K % 3], nvv,
                                                                              out + v0 * m, cnt);
        else
            k_gd_eval<<<grid_for(m, 1, kStreamGridCap), kBlock, 0, s>>>(g, t, owner, fv, gb[K % 3], nvv,
                                                                         out + v0 * m);
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

}  // extern "C"

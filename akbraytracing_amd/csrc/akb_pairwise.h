// numpy's pairwise summation as device building blocks (shared by akb_reduce.hip and
// akb_focus.hip). numpy's add.reduce over a contiguous float64 row sums each 8192-element buffer
// pairwise - a node of n > 128 elements splits at n2 = n/2 rounded down to a multiple of 8, a leaf
// of 8..128 elements keeps 8 running sums and returns ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) plus
// its tail, a leaf of < 8 elements is a plain left-to-right sum - and adds the buffers left to
// right.
#pragma once

#include "akb_common.h"

namespace akb {

constexpr int kPwLeaf = 128;
constexpr int kTreeLevels = 8;  // a buffer (<= 8192) has leaves down to depth 7, <= 64 per level

__device__ __forceinline__ int pw_split(int n) {
    int n2 = n / 2;
    return n2 - (n2 % 8);
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(b & 0xffffffffLL), l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ double nan_zero(double v, bool nan0, long long& cnt) {
    if (nan0 && v != v) return 0.0;
    ++cnt;
    return v;
}

// numpy pairwise leaf (n <= 128) over staged values (NaN already replaced)
// kNan0: read NaN as 0 (np.nansum's values) - the caller counts the non-NaN elements
template <bool kNan0 = false>
__device__ __forceinline__ double pw_val(const double* a, int i) {
    const double x = a[i];
    return (kNan0 && x != x) ? 0.0 : x;
}

template <bool kNan0 = false>
static __device__ double pw_leaf_lds(const double* a, int n) {
    if (n < 8) {
        double res = 0.0;
        for (int i = 0; i < n; ++i) res = res + pw_val<kNan0>(a, i);
        return res;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = pw_val<kNan0>(a, j);
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = r[j] + pw_val<kNan0>(a, i + j);
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res = res + pw_val<kNan0>(a, i);
    return res;
}

struct PwTree {
    int off[kTreeLevels][64];
    int len[kTreeLevels][64];
    int child[kTreeLevels][64];
    double val[kTreeLevels][64];
};

// numpy pairwise_sum of a[0..len), 0 < len < 8192, by one wave: the split tree is built top-down
// one level per step (a node of more than 128 elements splits at pw_split(n) into left and right
// children, placed in order by a ballot prefix count), each leaf is summed by one lane, and the
// levels are combined bottom-up as left + right.
template <bool kNan0 = false>
static __device__ double pw_tree_wave(PwTree& T, const double* a, int len) {
    const int lane = threadIdx.x & 63;
    if (lane == 0) {
        T.off[0][0] = 0;
        T.len[0][0] = len;
    }
    int nd[kTreeLevels];
    nd[0] = 1;
    int depth = 1;
    wave_sync();
#pragma unroll
    for (int d = 0; d < kTreeLevels; ++d) {
        if (d < depth) {
            const bool act = lane < nd[d];
            int o = 0, l = 0;
            if (act) {
                o = T.off[d][lane];
                l = T.len[d][lane];
            }
            const bool split = act && l > kPwLeaf && d + 1 < kTreeLevels;
            const unsigned long long m = __ballot(split);
            if (split) {
                const int pos = 2 * __popcll(m & ((1ull << lane) - 1ull));
                const int l2 = pw_split(l);
                if (d + 1 < kTreeLevels) {
                    T.off[d + 1][pos] = o;
                    T.len[d + 1][pos] = l2;
                    T.off[d + 1][pos + 1] = o + l2;
                    T.len[d + 1][pos + 1] = l - l2;
                }
                T.child[d][lane] = pos;
            } else if (act) {
                T.val[d][lane] = pw_leaf_lds<kNan0>(a + o, l);
            }
            if (m && d + 1 < kTreeLevels) {
                nd[d + 1] = 2 * __popcll(m);
                depth = d + 2;
            }
            wave_sync();
        }
    }
#pragma unroll
    for (int d = kTreeLevels - 2; d >= 0; --d) {
        if (d + 1 < depth) {
            if (lane < nd[d] && T.len[d][lane] > kPwLeaf) {
                const int c = T.child[d][lane];
                T.val[d][lane] = T.val[d + 1][c] + T.val[d + 1][c + 1];
            }
            wave_sync();
        }
    }
    return T.val[0][0];
}

// pw_leaf_lds / pw_tree_wave over a virtual array: get.leaf(o, n) is the numpy leaf sum of elements
// o .. o + n - 1 (8 running sums in order, as pw_leaf_lds), e.g. of a meshgrid's flattened entries
// formed from its axis; the same split tree and additions, so the same bits as the stored array's sum
template <class Get>
__device__ double pw_tree_wave_get(PwTree& T, const Get& get, int base, int len) {
    const int lane = threadIdx.x & 63;
    if (len == 64 * kPwLeaf) {
        // a full 8192-element buffer: numpy's split tree is balanced down to 64 leaves of 128 - a
        // leaf a lane, then the levels left + right as a butterfly in the tree's order (no tree
        // bookkeeping in LDS); every lane gets the root
        double v = get.leaf(base + kPwLeaf * lane, kPwLeaf);
        for (int off = 1; off < 64; off <<= 1) v = v + __shfl_down(v, off);
        return __shfl(v, 0);
    }
    if (lane == 0) {
        T.off[0][0] = 0;
        T.len[0][0] = len;
    }
    int nd[kTreeLevels];
    nd[0] = 1;
    int depth = 1;
    wave_sync();
#pragma unroll
    for (int d = 0; d < kTreeLevels; ++d) {
        if (d < depth) {
            const bool act = lane < nd[d];
            int o = 0, l = 0;
            if (act) {
                o = T.off[d][lane];
                l = T.len[d][lane];
            }
            const bool split = act && l > kPwLeaf && d + 1 < kTreeLevels;
            const unsigned long long m = __ballot(split);
            if (split) {
                const int pos = 2 * __popcll(m & ((1ull << lane) - 1ull));
                const int l2 = pw_split(l);
                T.off[d + 1][pos] = o;
                T.len[d + 1][pos] = l2;
                T.off[d + 1][pos + 1] = o + l2;
                T.len[d + 1][pos + 1] = l - l2;
                T.child[d][lane] = pos;
            } else if (act) {
                T.val[d][lane] = get.leaf(base + o, l);
            }
            if (m && d + 1 < kTreeLevels) {
                nd[d + 1] = 2 * __popcll(m);
                depth = d + 2;
            }
            wave_sync();
        }
    }
#pragma unroll
    for (int d = kTreeLevels - 2; d >= 0; --d) {
        if (d + 1 < depth) {
            if (lane < nd[d] && T.len[d][lane] > kPwLeaf) {
                const int c = T.child[d][lane];
                T.val[d][lane] = T.val[d + 1][c] + T.val[d + 1][c + 1];
            }
            wave_sync();
        }
    }
    return T.val[0][0];
}

// np.sum of a virtual contiguous float64 array of n elements by one wave: numpy's 8192-element
// buffers, each summed pairwise, added left to right
template <class Get>
__device__ double pw_sum_wave_get(PwTree& T, const Get& get, long long n) {
    double s = 0.0;
    bool first = true;
    for (long long b = 0; b < n; b += 8192) {
        const int len = (int)((n - b) < 8192 ? (n - b) : 8192);
        const double v = pw_tree_wave_get(T, get, (int)b, len);
        s = first ? v : s + v;
        first = false;
        wave_sync();
    }
    return s;
}

// the flattened my x mx meshgrid of an axis a as get.leaf wants it: element i is a[i % mx]
// (np.meshgrid's first output, rows) or a[i / mx] (its second, columns), walked in order
struct MeshgridAxis {
    const double* a;
    int mx;
    bool rows;
    __device__ double leaf(int o, int n) const {
        int r = o / mx, c = o - r * mx;
        auto next = [&]() {
            const double v = rows ? a[c] : a[r];
            if (++c == mx) {
                c = 0;
                ++r;
            }
            return v;
        };
        if (n < 8) {
            double res = 0.0;
            for (int i = 0; i < n; ++i) res = res + next();
            return res;
        }
        double acc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = next();
        int i = 8;
        for (; i < n - (n % 8); i += 8) {
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] = acc[j] + next();
        }
        double res = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
        for (; i < n; ++i) res = res + next();
        return res;
    }
};

}  // namespace akb

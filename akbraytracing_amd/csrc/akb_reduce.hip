// numpy-exact float64 row sums for gfx950 (np.sum / np.mean / np.nanmean of the drivers).
//
// numpy's add.reduce over a contiguous float64 row runs its inner loop on 8192-element buffers
// and adds the buffer results left to right; inside a buffer it uses pairwise_sum: a node of
// n > 128 elements splits at n2 = n/2 rounded down to a multiple of 8, a leaf of 8..128
// elements keeps 8 running sums r[j] += a[i+j] and returns ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7))
// plus the tail, and a leaf of < 8 elements is a plain left-to-right sum. Reproducing that order
// gives means bit-identical to the reference's (AKB_raytrace_20250312.py:3583-3591, :3626, :3633,
// :3674), which keeps the tilt angles and the OPD reference point exact.
//
// k_pw_chunks: one 256-thread workgroup per 8192-element buffer. The buffer is staged through LDS
// with coalesced loads (NaN -> 0 and the count happen here); leaves are laid out 136 doubles
// apart so the (leaf, accumulator) reads of a half-wave hit 64 distinct banks. A full buffer is
// always 64 leaves of 128: thread (leaf, j) runs accumulator j of its leaf, three xor-shuffles
// form the leaf in numpy's order, and one wave's six xor-shuffles form the exact split tree over
// the 64 leaves. The (at most one per row) short last buffer walks the generic split tree.
// k_pw_final adds the buffer results of a row left to right.
#include "akb_common.h"

namespace akb {

constexpr int kPwBuf = 8192;
constexpr int kPwLeaf = 128;
constexpr int kPwStride = 136;  // LDS doubles per leaf (128 + 8 padding)
constexpr int kPwThreads = 256;
constexpr int kPwMaxLeaves = 160;

__device__ __forceinline__ int pw_split(int n) {
    int n2 = n / 2;
    return n2 - (n2 % 8);
}

__device__ __forceinline__ double lds_at(const double* s, int idx) {
    return s[(idx >> 7) * kPwStride + (idx & (kPwLeaf - 1))];
}

// numpy pairwise leaf over staged elements [off, off + n)
__device__ double pw_leaf_lds(const double* s, int off, int n) {
    if (n < 8) {
        double res = 0.0;
        for (int i = 0; i < n; ++i) res = res + lds_at(s, off + i);
        return res;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = lds_at(s, off + j);
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = r[j] + lds_at(s, off + i + j);
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res = res + lds_at(s, off + i);
    return res;
}

// part / part_cnt: row r, buffer c lands at [r * part_ld + part_col0 + c]
__global__ void __launch_bounds__(kPwThreads) k_pw_chunks(const double* __restrict__ x, int64_t ld, int64_t n,
                                                          int nan_mask, int part_ld, int part_col0,
                                                          double* __restrict__ part,
                                                          long long* __restrict__ part_cnt) {
    __shared__ double s[(kPwBuf / kPwLeaf) * kPwStride];
    __shared__ double leafv[kPwMaxLeaves];
    __shared__ int leaf_off[kPwMaxLeaves], leaf_len[kPwMaxLeaves];
    __shared__ int n_leaves;
    __shared__ long long wcnt[kPwThreads / 64];
    const int row = blockIdx.y;
    const int c = blockIdx.x;
    const int tid = threadIdx.x;
    const double* a = x + row * ld + (int64_t)c * kPwBuf;
    const int64_t rem = n - (int64_t)c * kPwBuf;
    const int len = rem < kPwBuf ? (int)rem : kPwBuf;
    const bool nan0 = (nan_mask >> (row < 31 ? row : 31)) & 1;

    long long cnt = 0;
    // stage: 16 independent loads per thread in flight before the LDS stores (a full buffer is
    // 32 loads per thread, two batches)
    constexpr int kBatch = 16;
    for (int i0 = tid; i0 < len; i0 += kPwThreads * kBatch) {
        double v[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; ++k) {
            const int i = i0 + k * kPwThreads;
            v[k] = i < len ? a[i] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < kBatch; ++k) {
            const int i = i0 + k * kPwThreads;
            if (i < len) {
                double w = v[k];
                if (nan0 && w != w) {
                    w = 0.0;
                } else {
                    ++cnt;
                }
                s[(i >> 7) * kPwStride + (i & (kPwLeaf - 1))] = w;
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off);
    if ((tid & 63) == 0) wcnt[tid >> 6] = cnt;
    __syncthreads();

    double result;
    if (len == kPwBuf) {
        // 64 leaves x 8 accumulators = 512 sequences, two per thread
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int leaf = (tid >> 3) + 32 * h;
            const int j = tid & 7;
            const double* L = s + leaf * kPwStride + j;
            double r = L[0];
#pragma unroll
            for (int row8 = 1; row8 < kPwLeaf / 8; ++row8) r = r + L[row8 * 8];
            r = r + __shfl_xor(r, 1);
            r = r + __shfl_xor(r, 2);
            r = r + __shfl_xor(r, 4);
            if (j == 0) leafv[leaf] = r;
        }
        __syncthreads();
        if (tid < 64) {
            double v = leafv[tid];
            v = v + __shfl_xor(v, 1);
            v = v + __shfl_xor(v, 2);
            v = v + __shfl_xor(v, 4);
            v = v + __shfl_xor(v, 8);
            v = v + __shfl_xor(v, 16);
            v = v + __shfl_xor(v, 32);
            result = v;
        }
    } else {
        // short last buffer: enumerate the split tree's leaves, sum them in parallel, combine
        if (tid == 0) {
            int st_off[16], st_len[16];
            int sp = 1, nl = 0;
            st_off[0] = 0;
            st_len[0] = len;
            while (sp > 0) {
                --sp;
                const int o = st_off[sp], l = st_len[sp];
                if (l <= kPwLeaf) {
                    leaf_off[nl] = o;
                    leaf_len[nl] = l;
                    ++nl;
                } else {
                    const int l2 = pw_split(l);
                    st_off[sp] = o + l2;
                    st_len[sp] = l - l2;
                    ++sp;
                    st_off[sp] = o;
                    st_len[sp] = l2;
                    ++sp;
                }
            }
            n_leaves = nl;
        }
        __syncthreads();
        for (int li = tid; li < n_leaves; li += kPwThreads) leafv[li] = pw_leaf_lds(s, leaf_off[li], leaf_len[li]);
        __syncthreads();
        if (tid == 0) {
            // post-order evaluation of the same tree
            int st_len[16], st_state[16];
            double st_left[16];
            int sp = 1, li = 0;
            bool have = false;
            double res = 0.0;
            st_len[0] = len;
            st_state[0] = 0;
            while (sp > 0) {
                const int t = sp - 1;
                if (!have) {
                    if (st_len[t] <= kPwLeaf) {
                        res = leafv[li++];
                        have = true;
                        --sp;
                    } else {
                        st_state[t] = 1;
                        st_len[sp] = pw_split(st_len[t]);
                        st_state[sp] = 0;
                        ++sp;
                    }
                } else if (st_state[t] == 1) {
                    st_left[t] = res;
                    st_state[t] = 2;
                    have = false;
                    st_len[sp] = st_len[t] - pw_split(st_len[t]);
                    st_state[sp] = 0;
                    ++sp;
                } else {
                    res = st_left[t] + res;
                    --sp;
                }
            }
            result = res;
        }
    }
    if (tid == 0) {
        const int64_t o = (int64_t)row * part_ld + part_col0 + c;
        part[o] = result;
        long long tc = 0;
        for (int w = 0; w < kPwThreads / 64; ++w) tc += wcnt[w];
        part_cnt[o] = tc;
    }
}

// full 8192-element buffers from producer leaf sums: one wave per (buffer, quantity); the six
// xor-shuffles are numpy's split tree over the buffer's 64 leaves
__global__ void __launch_bounds__(64) k_leaf_chunks(const double* __restrict__ leaf_sum,
                                                    const int* __restrict__ leaf_cnt, int64_t nleaves,
                                                    int part_ld, double* __restrict__ part,
                                                    long long* __restrict__ part_cnt) {
    const int q = blockIdx.y;
    const int c = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t li = (int64_t)q * nleaves + (int64_t)c * 64 + lane;
    double v = leaf_sum[li];
    long long k = leaf_cnt[li];
    v = v + __shfl_xor(v, 1);
    v = v + __shfl_xor(v, 2);
    v = v + __shfl_xor(v, 4);
    v = v + __shfl_xor(v, 8);
    v = v + __shfl_xor(v, 16);
    v = v + __shfl_xor(v, 32);
    for (int off = 32; off > 0; off >>= 1) k += __shfl_down(k, off);
    if (lane == 0) {
        part[(int64_t)q * part_ld + c] = v;
        part_cnt[(int64_t)q * part_ld + c] = k;
    }
}

// one workgroup per row: buffer results added left to right (a single dependent chain, fed from
// LDS eight values ahead), counts summed by all threads
__global__ void __launch_bounds__(kPwThreads) k_pw_final(const double* __restrict__ part,
                                                         const long long* __restrict__ part_cnt, int nchunks,
                                                         double* __restrict__ out, int64_t* __restrict__ cnt_out) {
    constexpr int kTile = 4096;
    __shared__ double t[kTile];
    __shared__ long long wc[kPwThreads / 64];
    const int row = blockIdx.x;
    const int tid = threadIdx.x;
    const double* p = part + (int64_t)row * nchunks;
    const long long* pc = part_cnt + (int64_t)row * nchunks;
    long long cnt = 0;
    for (int i = tid; i < nchunks; i += kPwThreads) cnt += pc[i];
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off);
    if ((tid & 63) == 0) wc[tid >> 6] = cnt;
    double acc = 0.0;
    for (int base = 0; base < nchunks; base += kTile) {
        const int m = (nchunks - base) < kTile ? (nchunks - base) : kTile;
        __syncthreads();
        for (int i = tid; i < m; i += kPwThreads) t[i] = p[base + i];
        __syncthreads();
        if (tid == 0) {
            int i = 0;
            if (base == 0) {
                acc = t[0];
                i = 1;
            }
            for (; i + 8 <= m; i += 8) {
                double v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = t[i + k];
#pragma unroll
                for (int k = 0; k < 8; ++k) acc = acc + v[k];
            }
            for (; i < m; ++i) acc = acc + t[i];
        }
    }
    if (tid == 0) {
        out[row] = acc;
        long long tc = 0;
        for (int w = 0; w < kPwThreads / 64; ++w) tc += wc[w];
        cnt_out[row] = tc;
    }
}

}  // namespace akb

using namespace akb;

extern "C" {

int64_t akb_pairwise_work_bytes(int rows, int64_t n) {
    const int64_t nb = n <= 0 ? 1 : (n + kPwBuf - 1) / kPwBuf;
    return (int64_t)rows * nb * 16;
}

int akb_pairwise_sum_f64(const double* x, int64_t ld, int rows, int64_t n, int nan_to_zero, double* d_sum,
                         int64_t* d_count, void* d_work, void* stream) {
    clear_error();
    AKB_REQUIRE(x && d_sum && d_count && d_work, "null pointer");
    AKB_REQUIRE(rows > 0 && rows <= 65535 && n >= 0 && ld >= n, "bad sizes");
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        AKB_HIP_CHECK(hipMemsetAsync(d_count, 0, sizeof(int64_t) * rows, s));
        AKB_HIP_CHECK(hipMemsetAsync(d_sum, 0, sizeof(double) * rows, s));
        return AKB_OK;
    }
    const int64_t nb64 = (n + kPwBuf - 1) / kPwBuf;
    AKB_REQUIRE(nb64 < (1LL << 31), "row too long");
    const int nb = (int)nb64;
    double* part = (double*)d_work;
    long long* part_cnt = (long long*)(part + (int64_t)rows * nb);
    k_pw_chunks<<<dim3(nb, rows), kPwThreads, 0, s>>>(x, ld, n, nan_to_zero ? -1 : 0, nb, 0, part, part_cnt);
    int st = launch_status("k_pw_chunks");
    if (st) return st;
    k_pw_final<<<rows, kPwThreads, 0, s>>>(part, part_cnt, nb, d_sum, d_count);
    return launch_status("k_pw_final");
}

int64_t akb_leaf_sink_bytes(int nq, int64_t n) {
    if (nq <= 0 || n < 0) return 0;
    const int64_t nleaves = (n / kPwBuf) * (kPwBuf / kPwLeaf);
    const int64_t a = ((int64_t)nq * nleaves * 8 + 255) / 256 * 256;
    const int64_t b = ((int64_t)nq * nleaves * 4 + 255) / 256 * 256;
    return a + b + (int64_t)nq * kPwBuf * 8;
}

int akb_leaf_sink_layout(void* base, int nq, int nan_mask, int64_t n, akb_leaf_sink* out) {
    clear_error();
    AKB_REQUIRE(base && out && nq > 0 && nq <= 8 && n >= 0, "bad sink layout arguments");
    const int64_t nleaves = (n / kPwBuf) * (kPwBuf / kPwLeaf);
    const int64_t a = ((int64_t)nq * nleaves * 8 + 255) / 256 * 256;
    const int64_t b = ((int64_t)nq * nleaves * 4 + 255) / 256 * 256;
    out->leaf_sum = (double*)base;
    out->leaf_cnt = (int32_t*)((char*)base + a);
    out->tail = (double*)((char*)base + a + b);
    out->nq = nq;
    out->nan_mask = nan_mask;
    out->n = n;
    return AKB_OK;
}

int64_t akb_leaf_finish_work_bytes(int nq, int64_t n) {
    const int64_t nb = n <= 0 ? 1 : (n + kPwBuf - 1) / kPwBuf;
    return (int64_t)nq * nb * 16;
}

int akb_leaf_finish_f64(const akb_leaf_sink* sink, double* d_sum, int64_t* d_count, void* work, void* stream) {
    clear_error();
    AKB_REQUIRE(sink && d_sum && d_count && work, "null pointer");
    AKB_REQUIRE(sink->nq > 0 && sink->nq <= 8 && sink->n >= 0, "bad sink");
    hipStream_t s = (hipStream_t)stream;
    const int nq = sink->nq;
    if (sink->n == 0) {
        AKB_HIP_CHECK(hipMemsetAsync(d_count, 0, sizeof(int64_t) * nq, s));
        AKB_HIP_CHECK(hipMemsetAsync(d_sum, 0, sizeof(double) * nq, s));
        return AKB_OK;
    }
    const int64_t nfull = sink->n / kPwBuf;
    const int tail = (int)(sink->n - nfull * kPwBuf);
    const int nb = (int)(nfull + (tail > 0 ? 1 : 0));
    double* part = (double*)work;
    long long* part_cnt = (long long*)(part + (int64_t)nq * nb);
    int st;
    if (nfull > 0) {
        k_leaf_chunks<<<dim3((unsigned)nfull, nq), 64, 0, s>>>(sink->leaf_sum, sink->leaf_cnt,
                                                                nfull * (kPwBuf / kPwLeaf), nb, part, part_cnt);
        if ((st = launch_status("k_leaf_chunks"))) return st;
    }
    if (tail > 0) {
        k_pw_chunks<<<dim3(1, nq), kPwThreads, 0, s>>>(sink->tail, kPwBuf, tail, sink->nan_mask, nb,
                                                        (int)nfull, part, part_cnt);
        if ((st = launch_status("k_pw_chunks(tail)"))) return st;
    }
    k_pw_final<<<nq, kPwThreads, 0, s>>>(part, part_cnt, nb, d_sum, d_count);
    return launch_status("k_pw_final");
}

}  // extern "C"

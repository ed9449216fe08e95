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
// k_pw_chunks: one 256-thread workgroup per full 8192-element buffer. The buffer is staged
// through LDS with coalesced loads (NaN -> 0 and the count happen here); leaves are laid out 136
// doubles apart so the (leaf, accumulator) reads of a half-wave hit 64 distinct banks. A full
// buffer is always 64 leaves of 128: thread (leaf, j) runs accumulator j of its leaf, three
// xor-shuffles form the leaf in numpy's order, and one wave's six xor-shuffles form the exact
// split tree over the 64 leaves. k_leaf_chunks does the same from leaf sums a producer already
// formed. k_pw_final finishes a row: the buffer results added left to right, then the short last
// buffer's pairwise sum (its split tree built and combined level by level by one wave).
#include "akb_common.h"
#include "akb_pairwise.h"

namespace akb {

constexpr int kPwBuf = 8192;
constexpr int kPwStride = 136;  // LDS doubles per leaf (128 + 8 padding)
constexpr int kPwThreads = 256;
constexpr int kFinalTile = 4096;

// part / part_cnt: row r, buffer c lands at [r * part_ld + c]; only full buffers come here
__global__ void __launch_bounds__(kPwThreads) k_pw_chunks(const double* __restrict__ x, int64_t ld, int nan_mask,
                                                          int part_ld, double* __restrict__ part,
                                                          long long* __restrict__ part_cnt) {
    AKB_CHAIN_PRIORITY();
    __shared__ double s[(kPwBuf / kPwLeaf) * kPwStride];
    __shared__ double leafv[kPwBuf / kPwLeaf];
    __shared__ long long wcnt[kPwThreads / 64];
    const int row = blockIdx.y;
    const int c = blockIdx.x;
    const int tid = threadIdx.x;
    const double* a = x + row * ld + (int64_t)c * kPwBuf;
    const bool nan0 = (nan_mask >> (row < 31 ? row : 31)) & 1;

    long long cnt = 0;
    // stage: 16 independent loads per thread in flight before the LDS stores (32 loads per
    // thread, two batches)
    constexpr int kBatch = 16;
    for (int i0 = tid; i0 < kPwBuf; i0 += kPwThreads * kBatch) {
        double v[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; ++k) v[k] = a[i0 + k * kPwThreads];
#pragma unroll
        for (int k = 0; k < kBatch; ++k) {
            const int i = i0 + k * kPwThreads;
            s[(i >> 7) * kPwStride + (i & (kPwLeaf - 1))] = nan_zero(v[k], nan0, cnt);
        }
    }
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off);
    if ((tid & 63) == 0) wcnt[tid >> 6] = cnt;
    __syncthreads();

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
        if (tid == 0) {
            const int64_t o = (int64_t)row * part_ld + c;
            part[o] = v;
            long long tc = 0;
            for (int w = 0; w < kPwThreads / 64; ++w) tc += wcnt[w];
            part_cnt[o] = tc;
        }
    }
}

// full 8192-element buffers from producer leaf sums: one wave per (buffer, quantity); the six
// xor-shuffles are numpy's split tree over the buffer's 64 leaves
__global__ void __launch_bounds__(64) k_leaf_chunks(const double* __restrict__ leaf_sum,
                                                    const int* __restrict__ leaf_cnt, int64_t nleaves,
                                                    int part_ld, double* __restrict__ part,
                                                    long long* __restrict__ part_cnt) {
    AKB_CHAIN_PRIORITY();
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

// One workgroup per row q: the row's nparts full-buffer sums (part[q * part_ld + c]) added left to
// right by wave 0 (a single dependent chain fed lane by lane from an LDS tile of `tile` doubles),
// the short last buffer tail[q * tail_ld + 0 .. tail_len) staged to LDS and summed pairwise by wave
// 1 meanwhile, then added last. The LDS is sized to the row (dynamic: tile + tail_len doubles, 29
// KB for a 1e7-element row instead of a fixed 96 KB), so the kernel finds room on a CU beside a
// running trace kernel's workgroups instead of waiting for them to drain.
__global__ void __launch_bounds__(kPwThreads) k_pw_final(const double* __restrict__ part,
                                                         const long long* __restrict__ part_cnt, int part_ld,
                                                         int nparts, const double* __restrict__ tail,
                                                         int64_t tail_ld, int tail_len, int nan_mask,
                                                         double* __restrict__ out, int64_t* __restrict__ cnt_out,
                                                         int tile) {
    AKB_CHAIN_PRIORITY();
    extern __shared__ double dyn[];
    double* const t = dyn;
    double* const tl = dyn + tile;
    __shared__ PwTree T;
    __shared__ long long wc[kPwThreads / 64];
    __shared__ double tail_sum;
    const int q = blockIdx.x;
    const int tid = threadIdx.x;
    const int w = tid >> 6, lane = tid & 63;
    const bool nan0 = (nan_mask >> (q < 31 ? q : 31)) & 1;
    const double* p = part + (int64_t)q * part_ld;
    const long long* pc = part_cnt + (int64_t)q * part_ld;
    long long cnt = 0;
    {  // all count loads in flight at once (a latency chain otherwise)
        constexpr int kBatch = 8;
        for (int i0 = tid; i0 < nparts; i0 += kPwThreads * kBatch) {
            long long c[kBatch];
#pragma unroll
            for (int k = 0; k < kBatch; ++k) {
                const int i = i0 + k * kPwThreads;
                c[k] = i < nparts ? pc[i] : 0;
            }
#pragma unroll
            for (int k = 0; k < kBatch; ++k) cnt += c[k];
        }
    }
    {  // stage the short buffer: NaN -> 0 and the count here
        const double* a = tail + (int64_t)q * tail_ld;
        constexpr int kBatch = 8;
        for (int i0 = tid; i0 < tail_len; i0 += kPwThreads * kBatch) {
            double v[kBatch];
#pragma unroll
            for (int k = 0; k < kBatch; ++k) {
                const int i = i0 + k * kPwThreads;
                v[k] = i < tail_len ? a[i] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < kBatch; ++k) {
                const int i = i0 + k * kPwThreads;
                if (i < tail_len) tl[i] = nan_zero(v[k], nan0, cnt);
            }
        }
    }
    double acc = 0.0;
    for (int base = 0; base == 0 || base < nparts; base += tile) {
        const int m = nparts - base < tile ? nparts - base : tile;
        if (base > 0) __syncthreads();
        {
            constexpr int kBatch = kFinalTile / kPwThreads;  // the whole tile in one batch
            double v[kBatch];
#pragma unroll
            for (int k = 0; k < kBatch; ++k) {
                const int i = tid + k * kPwThreads;
                v[k] = i < m ? p[base + i] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < kBatch; ++k) {
                const int i = tid + k * kPwThreads;
                if (i < m) t[i] = v[k];
            }
        }
        __syncthreads();
        if (w == 0 && lane == 0 && m > 0) {
            // one lane walks the tile in order: 16 LDS reads in flight ahead of 16 dependent adds
            int i = 0;
            if (base == 0) {
                acc = t[0];
                i = 1;
            }
            double v[16], u[16];
            if (i + 16 <= m) {
#pragma unroll
                for (int k = 0; k < 16; ++k) v[k] = t[i + k];
            }
            for (; i + 32 <= m; i += 16) {
#pragma unroll
                for (int k = 0; k < 16; ++k) u[k] = t[i + 16 + k];
#pragma unroll
                for (int k = 0; k < 16; ++k) acc = acc + v[k];
#pragma unroll
                for (int k = 0; k < 16; ++k) v[k] = u[k];
            }
            if (i + 16 <= m) {
#pragma unroll
                for (int k = 0; k < 16; ++k) acc = acc + v[k];
                i += 16;
            }
            for (; i < m; ++i) acc = acc + t[i];
        }
        if (w == 1 && base == 0 && tail_len > 0) {
            const double v = pw_tree_wave(T, tl, tail_len);
            if (lane == 0) tail_sum = v;
        }
    }
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off);
    if (lane == 0) wc[w] = cnt;
    __syncthreads();
    if (tid == 0) {
        double r = acc;
        if (tail_len > 0) r = nparts > 0 ? acc + tail_sum : tail_sum;
        out[q] = r;
        long long tc = 0;
        for (int k = 0; k < kPwThreads / 64; ++k) tc += wc[k];
        cnt_out[q] = tc;
    }
}

// k_pw_final's part tile (at most kFinalTile doubles) and dynamic LDS bytes
static inline int final_tile(int nparts) { return nparts < 1 ? 1 : (nparts < kFinalTile ? nparts : kFinalTile); }
static inline size_t final_lds(int tile, int tail_len) { return (size_t)(tile + (tail_len > 0 ? tail_len : 1)) * 8; }

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
    const int64_t nfull = n / kPwBuf;
    const int tail = (int)(n - nfull * kPwBuf);
    double* part = (double*)d_work;
    long long* part_cnt = (long long*)(part + (int64_t)rows * nb);
    const int mask = nan_to_zero ? -1 : 0;
    if (nfull > 0) {
        k_pw_chunks<<<dim3((unsigned)nfull, rows), kPwThreads, 0, s>>>(x, ld, mask, nb, part, part_cnt);
        int st = launch_status("k_pw_chunks");
        if (st) return st;
    }
    const int tile = final_tile((int)nfull);
    k_pw_final<<<rows, kPwThreads, final_lds(tile, tail), s>>>(part, part_cnt, nb, (int)nfull, x + nfull * kPwBuf,
                                                              ld, tail, mask, d_sum, d_count, tile);
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
    AKB_REQUIRE(base && out && nq > 0 && nq <= 4096 && n >= 0, "bad sink layout arguments");
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
    AKB_REQUIRE(sink->nq > 0 && sink->nq <= 4096 && sink->n >= 0, "bad sink");
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
    if (nfull > 0) {
        k_leaf_chunks<<<dim3((unsigned)nfull, nq), 64, 0, s>>>(sink->leaf_sum, sink->leaf_cnt,
                                                                nfull * (kPwBuf / kPwLeaf), nb, part, part_cnt);
        int st = launch_status("k_leaf_chunks");
        if (st) return st;
    }
    const int tile = final_tile((int)nfull);
    k_pw_final<<<nq, kPwThreads, final_lds(tile, tail), s>>>(part, part_cnt, nb, (int)nfull, sink->tail, kPwBuf,
                                                            tail, sink->nan_mask, d_sum, d_count, tile);
    return launch_status("k_pw_final");
}

int akb_leaf_parts_f64(const akb_leaf_sink* sink, double* d_part, int64_t* d_part_cnt, int part_ld,
                       double* d_tail_sum, int64_t* d_tail_cnt, void* stream) {
    clear_error();
    AKB_REQUIRE(sink && d_part && d_part_cnt && d_tail_sum && d_tail_cnt, "null pointer");
    AKB_REQUIRE(sink->nq > 0 && sink->nq <= 4096 && sink->n >= 0, "bad sink");
    const int64_t nfull = sink->n / kPwBuf;
    const int tail = (int)(sink->n - nfull * kPwBuf);
    AKB_REQUIRE(part_ld >= nfull && part_ld >= 1, "part_ld below the sink's full buffers");
    hipStream_t s = (hipStream_t)stream;
    const int nq = sink->nq;
    if (nfull > 0) {
        k_leaf_chunks<<<dim3((unsigned)nfull, nq), 64, 0, s>>>(sink->leaf_sum, sink->leaf_cnt,
                                                                nfull * (kPwBuf / kPwLeaf), part_ld, d_part,
                                                                (long long*)d_part_cnt);
        int st = launch_status("k_leaf_chunks");
        if (st) return st;
    }
    if (tail == 0) {
        AKB_HIP_CHECK(hipMemsetAsync(d_tail_sum, 0, sizeof(double) * nq, s));
        AKB_HIP_CHECK(hipMemsetAsync(d_tail_cnt, 0, sizeof(int64_t) * nq, s));
        return AKB_OK;
    }
    // the short buffer alone: k_pw_final with no full buffers gives its pairwise sum and count
    k_pw_final<<<nq, kPwThreads, final_lds(1, tail), s>>>(d_part, (const long long*)d_part_cnt, part_ld, 0,
                                                         sink->tail, kPwBuf, tail, sink->nan_mask, d_tail_sum,
                                                         d_tail_cnt, 1);
    return launch_status("k_pw_final (tail)");
}

int akb_parts_chain_f64(const double* d_part, const int64_t* d_part_cnt, int part_ld, int nq, int nparts,
                        double* d_sum, int64_t* d_count, void* stream) {
    clear_error();
    AKB_REQUIRE(d_part && d_part_cnt && d_sum && d_count, "null pointer");
    AKB_REQUIRE(nq > 0 && nq <= 65535 && nparts >= 1 && part_ld >= nparts, "bad sizes");
    const int tile = final_tile(nparts);
    k_pw_final<<<nq, kPwThreads, final_lds(tile, 0), (hipStream_t)stream>>>(
        d_part, (const long long*)d_part_cnt, part_ld, nparts, nullptr, 0, 0, 0, d_sum, d_count, tile);
    return launch_status("k_pw_final (chain)");
}

}  // extern "C"

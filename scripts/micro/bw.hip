// HBM streaming microbenchmark: 8-B vs 16-B lanes, one vs several row streams, read:write mixes
// like the tilt (7 reads : 4 writes per ray) and OPD (4 : 2) kernels.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

template <int R, int W>
__global__ void __launch_bounds__(256) k_rows8(const double* __restrict__ in, double* __restrict__ out, long n, long ld) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        double s = 0.0;
#pragma unroll
        for (int r = 0; r < R; ++r) s += in[r * ld + i];
#pragma unroll
        for (int w = 0; w < W; ++w) out[w * ld + i] = s + w;
    }
}

template <int R, int W>
__global__ void __launch_bounds__(256) k_rows16(const double2* __restrict__ in, double2* __restrict__ out, long n2, long ld2) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n2; i += (long)gridDim.x * blockDim.x) {
        double2 s = make_double2(0.0, 0.0);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const double2 v = in[r * ld2 + i];
            s.x += v.x;
            s.y += v.y;
        }
#pragma unroll
        for (int w = 0; w < W; ++w) out[w * ld2 + i] = make_double2(s.x + w, s.y + w);
    }
}

template <typename F>
float timeit(F f) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    f();
    CHECK(hipEventRecord(a));
    for (int k = 0; k < 20; ++k) f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / 20;
}

int main() {
    const long n = 10004570;  // even, ~1e7 rays
    double *in, *out;
    CHECK(hipMalloc(&in, 8 * n * 8));
    CHECK(hipMalloc(&out, 8 * n * 8));
    CHECK(hipMemset(in, 0, 8 * n * 8));
    for (int grid : {2048, 4096, 8192, 16384}) {
#define RUN8(R, W)                                                                                  \
        {                                                                                           \
            float ms = timeit([&] { k_rows8<R, W><<<grid, 256>>>(in, out, n, n); });                \
            printf("8B  R=%d W=%d grid=%5d %7.1f us %5.2f TB/s\n", R, W, grid, ms * 1e3,            \
                   (R + W) * n * 8.0 / (ms * 1e-3) / 1e12);                                         \
        }
#define RUN16(R, W)                                                                                 \
        {                                                                                           \
            float ms = timeit([&] { k_rows16<R, W><<<grid, 256>>>((const double2*)in, (double2*)out, n / 2, n / 2); }); \
            printf("16B R=%d W=%d grid=%5d %7.1f us %5.2f TB/s\n", R, W, grid, ms * 1e3,            \
                   (R + W) * n * 8.0 / (ms * 1e-3) / 1e12);                                         \
        }
        RUN8(1, 1) RUN16(1, 1) RUN8(7, 4) RUN16(7, 4) RUN8(4, 2) RUN16(4, 2)
    }
    return 0;
}

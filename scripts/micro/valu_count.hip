// Counter calibration: kernels with a known number of wave-level VALU instructions of one kind, run
// under rocprofv3 --pmc to see how SQ_INSTS_VALU and the SQ_INSTS_VALU_*_F64 counters tally them
// (does a transcendental or a 64-bit move count once? does a compare?). Each kernel issues
// kReps x 16 instructions of its kind per wave, plus a handful of loop and store instructions.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/micro/valu_count scripts/micro/valu_count.hip
//   rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace -- scripts/micro/valu_count
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int kReps = 1000;
#define R16(X) X X X X X X X X X X X X X X X X

__global__ void k_fma(double* out, double a) {
    double x = a + threadIdx.x, y = 1.0000001, z = 1e-9;
    for (int i = 0; i < kReps; ++i) { R16(asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_mul(double* out, double a) {
    double x = a + threadIdx.x, y = 1.0000001;
    for (int i = 0; i < kReps; ++i) { R16(asm volatile("v_mul_f64 %0, %0, %1" : "+v"(x) : "v"(y));) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_rsq(double* out, double a) {
    double x = a + threadIdx.x;
    for (int i = 0; i < kReps; ++i) { R16(asm volatile("v_rsq_f64 %0, %0" : "+v"(x));) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_cmp(double* out, double a) {
    double x = a + threadIdx.x, y = 2.0;
    for (int i = 0; i < kReps; ++i) { R16(asm volatile("v_cmp_lt_f64 vcc, %0, %1" : : "v"(x), "v"(y) : "vcc");) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_mov64(double* out, double a) {
    double x = a + threadIdx.x, y;
    for (int i = 0; i < kReps; ++i) { R16(asm volatile("v_mov_b64 %0, %1" : "=v"(y) : "v"(x)); x = y;) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_divscale(double* out, double a) {
    double x = a + threadIdx.x, y = 3.0;
    for (int i = 0; i < kReps; ++i) { R16(asm volatile("v_div_scale_f64 %0, vcc, %0, %1, %0" : "+v"(x) : "v"(y) : "vcc");) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_cnd(double* out, double a) {
    unsigned x = threadIdx.x, y = 7;
    for (int i = 0; i < kReps; ++i) { R16(asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(y));) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_readlane(double* out, double a) {
    unsigned x = threadIdx.x;
    unsigned s;
    for (int i = 0; i < kReps; ++i) { R16(asm volatile("v_readlane_b32 %0, %1, 3" : "=s"(s) : "v"(x));) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x + s;
}

__global__ void k_fmac(double* out, double a) {
    double x = a + threadIdx.x, y = 1.0000001, z = 1e-9;
    for (int i = 0; i < kReps; ++i) { R16(asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_fixup(double* out, double a) {
    double x = a + threadIdx.x, y = 3.0, z = 0.5;
    for (int i = 0; i < kReps; ++i) { R16(asm volatile("v_div_fixup_f64 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_max(double* out, double a) {
    double x = a + threadIdx.x, y = 3.0;
    for (int i = 0; i < kReps; ++i) { R16(asm volatile("v_max_f64 %0, %0, %1" : "+v"(x) : "v"(y));) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_add(double* out, double a) {
    double x = a + threadIdx.x, y = 3.0;
    for (int i = 0; i < kReps; ++i) { R16(asm volatile("v_add_f64 %0, %0, %1" : "+v"(x) : "v"(y));) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main() {
    double* out;
    const int blocks = 1024, threads = 256;  // 4096 waves
    (void)hipMalloc(&out, sizeof(double) * blocks * threads);
    hipLaunchKernelGGL(k_fma, blocks, threads, 0, 0, out, 1.0);
    hipLaunchKernelGGL(k_mul, blocks, threads, 0, 0, out, 1.0);
    hipLaunchKernelGGL(k_rsq, blocks, threads, 0, 0, out, 1.0);
    hipLaunchKernelGGL(k_cmp, blocks, threads, 0, 0, out, 1.0);
    hipLaunchKernelGGL(k_mov64, blocks, threads, 0, 0, out, 1.0);
    hipLaunchKernelGGL(k_divscale, blocks, threads, 0, 0, out, 1.0);
    hipLaunchKernelGGL(k_cnd, blocks, threads, 0, 0, out, 1.0);
    hipLaunchKernelGGL(k_readlane, blocks, threads, 0, 0, out, 1.0);
    hipLaunchKernelGGL(k_fmac, blocks, threads, 0, 0, out, 1.0);
    hipLaunchKernelGGL(k_fixup, blocks, threads, 0, 0, out, 1.0);
    hipLaunchKernelGGL(k_max, blocks, threads, 0, 0, out, 1.0);
    hipLaunchKernelGGL(k_add, blocks, threads, 0, 0, out, 1.0);
    (void)hipDeviceSynchronize();
    printf("waves %d, instructions of the kind per wave %d\n", blocks * threads / 64, kReps * 16);
    (void)hipFree(out);
    return 0;
}

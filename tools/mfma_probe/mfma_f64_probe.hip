// fp64 throughput probe on MI355X: v_mfma_f64_16x16x4_f64 (independent accumulators, waves per
// SIMD 1/2) and v_fma_f64 (VALU), all CUs busy.  Prints TFLOP/s.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void mfma_loop(double* out, int iters) {
    d4 acc[NACC];
    for (int q = 0; q < NACC; ++q) acc[q] = d4{0, 0, 0, 0};
    double a = 1.0 + threadIdx.x * 1e-9, b = 0.5 + blockIdx.x * 1e-9;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int q = 0; q < NACC; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
    }
    double s = 0;
    for (int q = 0; q < NACC; ++q) s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void fma_loop(double* out, int iters) {
    double x[8];
    for (int q = 0; q < 8; ++q) x[q] = threadIdx.x * 1e-9 + q;
    const double m = 0.999999, c = 1e-7;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int q = 0; q < 8; ++q) x[q] = __builtin_fma(x[q], m, c);
    }
    double s = 0;
    for (int q = 0; q < 8; ++q) s += x[q];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    double* d;
    hipMalloc(&d, sizeof(double) * 1024 * 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 20000;
    for (int wps : {1, 2}) {                         // waves per SIMD
        const int threads = 256 * wps, blocks = 256;
        hipLaunchKernelGGL(mfma_loop<8>, dim3(blocks), dim3(threads), 0, 0, d, 100);
        hipEventRecord(e0);
        hipLaunchKernelGGL(mfma_loop<8>, dim3(blocks), dim3(threads), 0, 0, d, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double flops = 2.0 * 16 * 16 * 4 * 8 * (double)iters * (threads / 64) * blocks;
        printf("mfma_f64_16x16x4 x8 acc, %d wave(s)/SIMD: %.2f TFLOP/s (%.3f ms)\n", wps,
               flops / ms / 1e9, ms);
    }
    for (int wps : {1, 2, 4}) {
        const int threads = 256 * wps, blocks = 256;
        hipLaunchKernelGGL(fma_loop, dim3(blocks), dim3(threads), 0, 0, d, 100);
        hipEventRecord(e0);
        hipLaunchKernelGGL(fma_loop, dim3(blocks), dim3(threads), 0, 0, d, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double flops = 2.0 * 8 * (double)iters * threads * blocks;
        printf("v_fma_f64 x8 chains, %d wave(s)/SIMD: %.2f TFLOP/s (%.3f ms)\n", wps,
               flops / ms / 1e9, ms);
    }
    return 0;
}

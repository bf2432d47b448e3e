// VALU issue / dependent latency of f64 (and f32, int) ops on one SIMD: a single workgroup of
// W waves (W = 1..4 per SIMD when launched with 4W waves), each running C independent chains of
// N dependent operations; prints cycles per operation per wave.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int C>
__global__ void chain_add_f64(double* out, double y, int n, long long* cyc) {
    double x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = threadIdx.x + c;
    __syncthreads();
    const long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
#pragma unroll
            for (int c = 0; c < C; ++c) asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[c]) : "v"(y));
        }
    }
    const long long t1 = __builtin_readcyclecounter();
    double s = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[threadIdx.x >> 6] = t1 - t0;
}

template <int C>
__global__ void chain_fma_f64(double* out, double y, int n, long long* cyc) {
    double x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = threadIdx.x + c;
    __syncthreads();
    const long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
#pragma unroll
            for (int c = 0; c < C; ++c) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(x[c]) : "v"(y));
        }
    }
    const long long t1 = __builtin_readcyclecounter();
    double s = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[threadIdx.x >> 6] = t1 - t0;
}

template <int C>
__global__ void chain_add_f32(double* out, double y, int n, long long* cyc) {
    float x[C];
    const float yf = (float)y;
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = threadIdx.x + c;
    __syncthreads();
    const long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
#pragma unroll
            for (int c = 0; c < C; ++c) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[c]) : "v"(yf));
        }
    }
    const long long t1 = __builtin_readcyclecounter();
    double s = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[threadIdx.x >> 6] = t1 - t0;
}

template <class K>
static void run(const char* name, K k, int waves_per_simd, double* out, long long* cyc) {
    const int n = 2000;
    const int threads = 64 * 4 * waves_per_simd;
    hipLaunchKernelGGL(k, dim3(1), dim3(threads), 0, 0, out, 1e-9, n, cyc);   // warm
    hipLaunchKernelGGL(k, dim3(1), dim3(threads), 0, 0, out, 1e-9, n, cyc);
    hipDeviceSynchronize();
    long long h[64];
    hipMemcpy(h, cyc, sizeof(long long) * 4 * waves_per_simd, hipMemcpyDeviceToHost);
    double m = 0;
    for (int w = 0; w < 4 * waves_per_simd; ++w) m += (double)h[w];
    m /= 4 * waves_per_simd;
    printf("%-14s waves/SIMD %d: %.2f cycles per instruction per wave\n", name, waves_per_simd,
           m / (n * 16.0));
}

int main() {
    double* out;
    long long* cyc;
    hipMalloc(&out, 8 * 4096);
    hipMalloc(&cyc, 8 * 64);
    for (int w = 1; w <= 3; ++w) {
        run("add_f64 x1", chain_add_f64<1>, w, out, cyc);
        run("add_f64 x2", chain_add_f64<2>, w, out, cyc);
        run("add_f64 x4", chain_add_f64<4>, w, out, cyc);
        run("fma_f64 x1", chain_fma_f64<1>, w, out, cyc);
        run("fma_f64 x4", chain_fma_f64<4>, w, out, cyc);
        run("add_f32 x1", chain_add_f32<1>, w, out, cyc);
        run("add_f32 x4", chain_add_f32<4>, w, out, cyc);
    }
    return 0;
}

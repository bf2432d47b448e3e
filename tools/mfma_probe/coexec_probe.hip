// Co-execution probe on MI355X: one 512-thread workgroup per CU (two waves per SIMD).  Waves 0-3
// run role A, waves 4-7 role B; each wave times its own loop with s_memtime.  Roles:
//   0 idle, 1 f64 MFMA 16x16x4 (8 independent accumulators), 2 v_fma_f64 (8 chains),
//   3 v_fma_f32 (8 chains), 4 v_add_u32 (8 chains), 5 ds_write_b64 (stream into LDS),
//   6 global loads (512 B per wave per load, streamed from a large buffer)
// Prints per role the average cycles per loop iteration, alone and paired.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double run_role(int role, int iters, const double* src, size_t nsrc,
                                           double* lds) {
    const int lane = threadIdx.x & 63;
    double sink = 0.0;
    if (role == 1) {
        d4 acc[8];
        for (int q = 0; q < 8; ++q) acc[q] = d4{0, 0, 0, 0};
        double a = 1.0 + lane * 1e-9, b = 0.5;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int q = 0; q < 8; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
        }
        for (int q = 0; q < 8; ++q) sink += acc[q][0];
    } else if (role == 2) {
        double x[8];
        for (int q = 0; q < 8; ++q) x[q] = lane * 1e-9 + q;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int q = 0; q < 8; ++q) x[q] = __builtin_fma(x[q], 0.999999, 1e-7);
        }
        for (int q = 0; q < 8; ++q) sink += x[q];
    } else if (role == 3) {
        float x[8];
        for (int q = 0; q < 8; ++q) x[q] = lane * 1e-6f + q;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int q = 0; q < 8; ++q) x[q] = __builtin_fmaf(x[q], 0.999f, 1e-3f);
        }
        for (int q = 0; q < 8; ++q) sink += x[q];
    } else if (role == 4) {
        unsigned x[8];
        for (int q = 0; q < 8; ++q) x[q] = lane + q;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int q = 0; q < 8; ++q) { x[q] = x[q] + (unsigned)i; asm volatile("" : "+v"(x[q])); }
        }
        for (int q = 0; q < 8; ++q) sink += x[q];
    } else if (role == 5) {
        const int w = (threadIdx.x >> 6) & 3;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int q = 0; q < 8; ++q) lds[(w * 8 + q) * 64 + lane] = (double)i;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    } else if (role == 6) {
        const size_t base = ((size_t)blockIdx.x * 4 + ((threadIdx.x >> 6) & 3)) * 64 * 8 * 64;
        double acc = 0.0;
        for (int i = 0; i < iters; ++i) {
            double v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = src[(base + ((size_t)(i & 63) * 8 + q) * 64 + lane) % nsrc];
#pragma unroll
            for (int q = 0; q < 8; ++q) acc += v[q];
        }
        sink += acc;
    }
    return sink;
}

__global__ __launch_bounds__(512) void coexec(int ra, int rb, int iters, const double* src,
                                              size_t nsrc, double* out, long long* cyc) {
    __shared__ double lds[32 * 64];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int role = wave < 4 ? ra : rb;
    __syncthreads();
    const long long t0 = __builtin_readcyclecounter();
    const double s = run_role(role, iters, src, nsrc, lds);
    const long long t1 = __builtin_readcyclecounter();
    out[blockIdx.x * 512 + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}

int main() {
    const size_t nsrc = (size_t)1 << 28;               // 2 GiB of doubles
    double *src, *out;
    long long* cyc;
    hipMalloc(&src, nsrc * sizeof(double));
    hipMemset(src, 0, nsrc * sizeof(double));
    hipMalloc(&out, sizeof(double) * 256 * 512);
    hipMalloc(&cyc, sizeof(long long) * 256 * 8);
    static long long h[256 * 8];
    const char* names[] = {"idle", "mfma_f64", "fma_f64", "fma_f32", "add_u32", "ds_write", "gload"};
    const int iters = 4000;
    auto run = [&](int ra, int rb, double* ca, double* cb) {
        hipLaunchKernelGGL(coexec, dim3(256), dim3(512), 0, 0, ra, rb, iters, src, nsrc, out, cyc);
        hipDeviceSynchronize();
        hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        double sa = 0, sb = 0;
        for (int b = 0; b < 256; ++b)
            for (int w = 0; w < 8; ++w) (w < 4 ? sa : sb) += h[b * 8 + w];
        *ca = sa / 1024.0 / iters;
        *cb = sb / 1024.0 / iters;
    };
    double a, b;
    run(1, 0, &a, &b);
    const double mf_alone = a;
    printf("mfma_f64 alone: %.1f cyc/iter (8 MFMAs)\n", a);
    for (int rb = 2; rb <= 6; ++rb) {
        double ba, bb;
        run(0, rb, &ba, &bb);
        run(1, rb, &a, &b);
        printf("%-9s alone %7.1f cyc/iter | paired with mfma_f64: %-9s %7.1f, mfma %7.1f (alone %.1f)\n",
               names[rb], bb, names[rb], b, a, mf_alone);
    }
    return 0;
}

// Read-order probe (round 5): the pooled Gram's producers stream 98 factor planes [T][lda] in
// 512-B segments (64 assets x 8 B) -- per workgroup item one 64-asset row-block over a chunk of 64
// dates, so consecutive loads of a plane are lda * 8 B apart and each touches another DRAM page.
// This probe times the bare read stream (8 producer-like waves per workgroup, one workgroup per CU,
// two row-blocks of loads in flight per wave, values folded into a sink) for items of
// G row-blocks x D dates (G * D = 64 row-block-dates), dates outer, row-blocks inner.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kP = 98, kWaves = 8, kMC = (kP + kWaves - 1) / kWaves;   // 13 planes per wave

template <int G>
__global__ __launch_bounds__(512, 1) void probe(const double* base, long long cs, int lda, int T,
                                                int nrb, double* sink) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr int D = 64 / G;
    const int ngrp = nrb / G, nch = (T + D - 1) / D, nitems = ngrp * nch;
    double acc = 0.0;
    for (int it = blockIdx.x; it < nitems; it += gridDim.x) {
        const int g = it / nch, c = it - g * nch;
        const int t0 = c * D, t1 = t0 + D < T ? t0 + D : T;
        double a[kMC], b[kMC];
        auto ld = [&](int k, double (&v)[kMC]) {
            const int t = t0 + k / G, rb = g * G + k % G;
            const long long off = (long long)t * lda + rb * 64 + lane;
#pragma unroll
            for (int j = 0; j < kMC; ++j) {
                const int pl = w + kWaves * j < kP ? w + kWaves * j : kP - 1;
                v[j] = base[pl * cs + off];
            }
        };
        const int n = (t1 - t0) * G;
        ld(0, a);
        for (int k = 0; k < n; k += 2) {
            ld(k + 1 < n ? k + 1 : k, b);
#pragma unroll
            for (int j = 0; j < kMC; ++j) acc += a[j];
            ld(k + 2 < n ? k + 2 : k, a);
#pragma unroll
            for (int j = 0; j < kMC; ++j) acc += b[j];
        }
    }
    sink[blockIdx.x * 512 + threadIdx.x] = acc;
}

template <int G>
float run(const double* base, long long cs, int lda, int T, double* sink, int grid) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    probe<G><<<grid, 512>>>(base, cs, lda, T, lda / 64, sink);
    hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) probe<G><<<grid, 512>>>(base, cs, lda, T, lda / 64, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 3;
}


// FM-like stream: NPL planes (NPL / 8 per wave), DEPTH row-blocks of loads in flight per wave
template <int NPL, int DEPTH>
__global__ __launch_bounds__(512, 1) void probe_fm(const double* base, long long cs, int lda, int T,
                                                   int nrb, double* sink) {
    constexpr int MC = NPL / kWaves;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nch = (T + 63) / 64, nitems = nrb * nch;
    double acc = 0.0;
    for (int it = blockIdx.x; it < nitems; it += gridDim.x) {
        const int g = it / nch, c = it - g * nch;
        const int t0 = c * 64, t1 = t0 + 64 < T ? t0 + 64 : T;
        const int n = t1 - t0;
        double v[DEPTH][MC];
        auto ld = [&](int k, double (&x)[MC]) {
            const int t = t0 + (k < n ? k : n - 1);
            const long long off = (long long)t * lda + g * 64 + lane;
#pragma unroll
            for (int j = 0; j < MC; ++j) x[j] = base[(w + kWaves * j) * cs + off];
        };
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) ld(d, v[d]);
        for (int k = 0; k < n; k += DEPTH) {
#pragma unroll
            for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
                for (int j = 0; j < MC; ++j) acc += v[d][j];
                ld(k + d + DEPTH, v[d]);
            }
        }
    }
    sink[blockIdx.x * 512 + threadIdx.x] = acc;
}

template <int NPL, int DEPTH>
float run_fm(const double* base, long long cs, int lda, int T, double* sink, int grid) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    probe_fm<NPL, DEPTH><<<grid, 512>>>(base, cs, lda, T, lda / 64, sink);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) probe_fm<NPL, DEPTH><<<grid, 512>>>(base, cs, lda, T, lda / 64, sink);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 3;
}

int main(int argc, char** argv) {
    const int lda = argc > 1 ? atoi(argv[1]) : 10240, T = argc > 2 ? atoi(argv[2]) : 4032;
    const long long cs = (long long)T * lda;
    double *base, *sink;
    if (hipMalloc(&base, sizeof(double) * cs * kP) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(base, 0, sizeof(double) * cs * kP);
    hipMalloc(&sink, sizeof(double) * 512 * 4096);
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const double gb = (double)cs * kP * 8 / 1e9;
    printf("planes %d x [%d][%d], %.2f GB per pass, grid %d x 512\n", kP, T, lda, gb, ncu);
    const double gb32 = (double)cs * 32 * 8 / 1e9;
    for (int rep = 0; rep < 2; ++rep) {
        float ms;
        ms = run_fm<32, 2>(base, cs, lda, T, sink, ncu);  printf("FM-like 32 planes, 2 row-blocks in flight: %7.3f ms %6.2f TB/s\n", ms, gb32 / ms);
        ms = run_fm<32, 4>(base, cs, lda, T, sink, ncu);  printf("FM-like 32 planes, 4 in flight:            %7.3f ms %6.2f TB/s\n", ms, gb32 / ms);
        ms = run_fm<32, 8>(base, cs, lda, T, sink, ncu);  printf("FM-like 32 planes, 8 in flight:            %7.3f ms %6.2f TB/s\n", ms, gb32 / ms);
        ms = run_fm<32, 2>(base, cs, lda, T, sink, 2 * ncu);  printf("FM-like 32 planes, 2 in flight, 2 WG/CU:   %7.3f ms %6.2f TB/s\n", ms, gb32 / ms);
    }
    for (int rep = 0; rep < 1; ++rep) {
        float ms;
        ms = run<1>(base, cs, lda, T, sink, ncu);  printf("G=1  (1 row-block x 64 dates): %7.3f ms %6.2f TB/s\n", ms, gb / ms);
        ms = run<2>(base, cs, lda, T, sink, ncu);  printf("G=2  (2 x 32):                %7.3f ms %6.2f TB/s\n", ms, gb / ms);
        ms = run<4>(base, cs, lda, T, sink, ncu);  printf("G=4  (4 x 16):                %7.3f ms %6.2f TB/s\n", ms, gb / ms);
        ms = run<8>(base, cs, lda, T, sink, ncu);  printf("G=8  (8 x 8):                 %7.3f ms %6.2f TB/s\n", ms, gb / ms);
        ms = run<16>(base, cs, lda, T, sink, ncu); printf("G=16 (16 x 4):                %7.3f ms %6.2f TB/s\n", ms, gb / ms);
        ms = run<1>(base, cs, lda, T, sink, 2 * ncu);  printf("G=1, 2 WG/CU grid:            %7.3f ms %6.2f TB/s\n", ms, gb / ms);
    }
    return 0;
}

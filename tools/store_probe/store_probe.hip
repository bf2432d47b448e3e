// Store-pattern probe for the factor kernel: the same grid (236 workgroups of two
// 6-wave items at config C: 5 job waves + 1 reader wave per item, 3 items per 64-asset block),
// the same 8-day chunks with a barrier each, the same output rows (96 planes [T][lda], every job
// wave storing its ~6-7 columns as 512-B rows per day) -- but no factor arithmetic.  Measures the
// time the output stream alone needs in that pattern.
//   hipcc -O3 --offload-arch=gfx950 tools/store_probe/store_probe.hip -o tools/store_probe/store_probe
//   ./store_probe [T=5040] [A=10000] [mode] [pad doubles between planes]   mode 0: stores+barriers, 1: stores only, 2: reads only;
//   +4: nontemporal stores; +8: block-major planes; 16 / 17: a plain / nontemporal 16-B
//   store stream over the planes; 18 / 19: an 8-B store stream, 1024 x 256 / the factor grid]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int kChunk = 8, kPlanes = 96;

__global__ __launch_bounds__(768) void probe(double* out, const double* in, long T, long lda,
                                             int nblk, int mode, long pad, int G, int work) {
    const int lane = threadIdx.x & 63, wall = threadIdx.x >> 6;
    const int half = wall >= 6 ? 1 : 0, pos = wall - 6 * half;
    const long item = 2L * blockIdx.x + half;
    const int type = (int)(item / nblk);
    const long block = item % nblk;
    const bool live = item < 3L * nblk;
    const long asset = block * 64 + lane;
    // job wave j of type t owns columns [c0, c1) of the 96 (15 sets, 6 or 7 columns each)
    const int set = type * 5 + pos;
    const int c0 = set * 96 / 15, c1 = (set + 1) * 96 / 15;
    const long plane = T * lda + pad;          // pad: extra doubles between consecutive planes
    double acc = 0.0;
    for (long ch = 0; ch * kChunk < T; ++ch) {
        if (live && pos < 5 && (mode & 3) != 2 && (mode & 64)) {
            // +64: column-pair planes [48][T][lda][2]: one 16-B store per lane = two columns of
            // one asset-day, 1 KB contiguous per instruction
            typedef double dv2 __attribute__((ext_vector_type(2)));
            for (int s = 0; s < kChunk; ++s) {
                const long t = ch * kChunk + s;
                if (t >= T) break;
                for (int c = c0 & ~1; c < c1; c += 2) {
                    const long off = (c >> 1) * 2 * plane + 2 * (t * lda + asset);
                    const dv2 v = {(double)t, (double)c};
                    *(dv2*)&out[off] = v;
                }
            }
        } else if (live && pos < 5 && (mode & 3) != 2 && (mode & 128)) {
            // +128: 16-B stores, two columns per instruction (even lanes: column c of assets
            // 2i, 2i+1; odd lanes: column c + 1 of the same two assets)
            typedef double dv2 __attribute__((ext_vector_type(2)));
            for (int s = 0; s < kChunk; ++s) {
                const long t = ch * kChunk + s;
                if (t >= T) break;
                for (int c = c0; c < c1; c += 2) {
                    const int cc = (lane & 1) && c + 1 < c1 ? c + 1 : c;
                    const long off = cc * plane + t * lda + block * 64 + (lane & ~1);
                    const dv2 v = {(double)t, (double)cc};
                    if ((lane & 1) == 0 || c + 1 < c1) *(dv2*)&out[off] = v;
                }
            }
        } else if (live && pos < 5 && (mode & 3) != 2 && (mode & 32)) {
            // +32: a column's days stored back to back, in groups of G days of the chunk
            for (int g0 = 0; g0 < kChunk; g0 += G)
            for (int c = c0; c < c1; ++c) {
                for (int s = g0; s < g0 + G; ++s) {
                    const long t = ch * kChunk + s;
                    if (t >= T) break;
                    const long off = (mode & 8) ? c * plane + block * (T * 64) + t * 64 + lane
                                                : c * plane + t * lda + asset;
                    // `work` f64 FMAs on 4 independent chains per stored value (compute beside
                    // the stores, as in the factor kernel)
                    double v0 = (double)t + c, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3;
                    for (int w = 0; w < work; w += 4) {
                        v0 = __builtin_fma(v0, 1.0000001, 0.5); v1 = __builtin_fma(v1, 1.0000001, 0.5);
                        v2 = __builtin_fma(v2, 1.0000001, 0.5); v3 = __builtin_fma(v3, 1.0000001, 0.5);
                    }
                    out[off] = v0 + v1 + v2 + v3;
                }
            }
        } else if (live && pos < 5 && (mode & 3) != 2) {
            for (int s = 0; s < kChunk; ++s) {
                const long t = ch * kChunk + s;
                if (t >= T) break;
                for (int c = c0; c < c1; ++c) {
                    // +8: block-major planes [lda / 64][T][64] (a block's dates contiguous)
                    const long off = (mode & 8) ? c * plane + block * (T * 64) + t * 64 + lane
                                                : c * plane + t * lda + asset;
                    if (mode & 4) __builtin_nontemporal_store((double)t + c, &out[off]);
                    else out[off] = (double)t + c;
                }
            }
        } else if (live && pos == 5) {
            for (int s = 0; s < kChunk; ++s) {
                const long t = ch * kChunk + s;
                if (t < T) acc += in[t * lda + asset] + in[plane / kPlanes * 0 + (T + t) * lda + asset];
            }
        }
        if ((mode & 3) != 1) __syncthreads();
    }
    if (acc == 12345.0) out[asset] = acc;
}

// the write ceiling: a grid-stride stream of 8-B stores over the same 96 planes
__global__ __launch_bounds__(768) void stream8(double* out, long n) {
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = (double)i;
}
// ... of 16-B stores
typedef double dv2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void stream(dv2* out, long n, int nt) {
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const dv2 v = {(double)i, 1.0};
        if (nt) __builtin_nontemporal_store(v, &out[i]);
        else out[i] = v;
    }
}

int main(int argc, char** argv) {
    const long T = argc > 1 ? atol(argv[1]) : 5040, A = argc > 2 ? atol(argv[2]) : 10000;
    const int mode = argc > 3 ? atoi(argv[3]) : 0;
    const long pad = argc > 4 ? atol(argv[4]) : 0;
    const int G = argc > 5 ? atoi(argv[5]) : kChunk;
    const int work = argc > 6 ? atoi(argv[6]) : 0;      // f64 FMAs per stored value (mode 32)
    const long lda = (A + 63) / 64 * 64;
    const int nblk = (int)(lda / 64);
    double *out, *in;
    if (hipMalloc(&out, sizeof(double) * kPlanes * (T * lda + pad)) != hipSuccess) return 1;
    if (hipMalloc(&in, sizeof(double) * 2 * T * lda) != hipSuccess) return 1;
    hipMemset(in, 0, sizeof(double) * 2 * T * lda);
    const int grid = (3 * nblk + 1) / 2;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int r = 0; r < 6; ++r) {
        hipEventRecord(e0);
        if (mode == 18)            // 18: 8-B streaming stores, 16 waves per CU
            hipLaunchKernelGGL(stream8, dim3(1024), dim3(256), 0, 0, out, (long)kPlanes * T * lda);
        else if (mode == 19)       // 19: 8-B streaming stores, the factor kernel's grid (12-wave WGs)
            hipLaunchKernelGGL(stream8, dim3(grid), dim3(768), 0, 0, out, (long)kPlanes * T * lda);
        else if (mode >= 16)       // 16 / 17: plain / nontemporal streaming stores
            hipLaunchKernelGGL(stream, dim3(4096), dim3(256), 0, 0, (dv2*)out,
                               (long)kPlanes * T * lda / 2, mode & 1);
        else
            hipLaunchKernelGGL(probe, dim3(grid), dim3(768), 0, 0, out, in, T, lda, nblk, mode, pad, G, work);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double gb = ((mode & 3) == 2 ? 16.0 : 8.0 * kPlanes) * T * A / 1e9;
        printf("work %d mode %d G %d T %ld A %ld pad %ld: %.3f ms  %.2f GB  %.2f TB/s\n", work, mode, G, T, A, pad, ms, gb,
               gb / ms);
    }
    return 0;
}

// Which SIMD does wave w of a workgroup issue on?  Launches one workgroup per CU (large dynamic
// LDS) of W waves and records HW_ID.SIMD_ID of every wave; prints, per wave index, how often each
// SIMD was seen.  Usage: simd_probe [waves=13]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void probe(int* out) {
    extern __shared__ double lds[];
    const int wave = threadIdx.x >> 6;
    // HW_ID (hwreg 4): SIMD_ID = bits [5:4]
    const int hw = __builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4);
    if ((threadIdx.x & 63) == 0) {
        lds[wave] = hw;
        out[blockIdx.x * 16 + wave] = hw & 3;
    }
}

int main(int argc, char** argv) {
    const int waves = argc > 1 ? atoi(argv[1]) : 13;
    const int nwg = 512;
    int* d = nullptr;
    hipMalloc(&d, sizeof(int) * nwg * 16);
    hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    hipLaunchKernelGGL(probe, dim3(nwg), dim3(64 * waves), 150 * 1024, 0, d);
    hipDeviceSynchronize();
    std::vector<int> h(nwg * 16);
    hipMemcpy(h.data(), d, sizeof(int) * nwg * 16, hipMemcpyDeviceToHost);
    printf("waves=%d: count of workgroups where wave w ran on SIMD s\n", waves);
    for (int w = 0; w < waves; ++w) {
        int c[4] = {0, 0, 0, 0};
        for (int b = 0; b < nwg; ++b) c[h[b * 16 + w] & 3]++;
        printf("wave %2d: %4d %4d %4d %4d\n", w, c[0], c[1], c[2], c[3]);
    }
    int same = 0;
    for (int b = 0; b < nwg; ++b) {
        bool ok = true;
        for (int w = 0; w < waves; ++w) ok = ok && ((h[b * 16 + w] - h[b * 16]) & 3) == (w & 3);
        same += ok;
    }
    printf("workgroups whose wave w sits on SIMD (simd(wave0) + w) %% 4: %d / %d\n", same, nwg);
    hipFree(d);
    return 0;
}

// LDS co-residency probe: how many workgroups of a given LDS size does one CU hold at once?
// Each workgroup records its CU (XCC/SE/CU ids) and [start, end) on the 100 MHz realtime clock
// while spinning ~40 us; the host counts the maximum overlap per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>
#include <algorithm>

template <int V>
__global__ void probe(long long* rec, int spin_ticks) {
    extern __shared__ double buf[];
    if (V == 1) asm volatile("" ::: "v118");         // force a 119-VGPR allocation
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    buf[threadIdx.x] = (double)threadIdx.x;          // touch the allocation
    long long t = t0;
    while (t - t0 < spin_ticks) t = (long long)__builtin_amdgcn_s_memrealtime();
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
        unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11)); // HW_REG_XCC_ID
        rec[blockIdx.x * 4 + 0] = t0;
        rec[blockIdx.x * 4 + 1] = t;
        rec[blockIdx.x * 4 + 2] = hw;
        rec[blockIdx.x * 4 + 3] = xcc + 0.0 * buf[threadIdx.x + 1];
    }
}

int main(int argc, char** argv) {
    const int nwg = 2048;
    const int threads = argc > 1 ? atoi(argv[1]) : 256;
    const int vg = argc > 2 ? atoi(argv[2]) : 0;      // 1: 119 VGPRs per wave
    long long* d;
    hipMalloc(&d, sizeof(long long) * 4 * nwg);
    std::vector<long long> h(4 * nwg);
    int sizes[] = {32768, 40960, 49152, 51200, 52224, 53248, 54272, 55296, 57344, 65536, 73728, 78336, 81920};
    for (int lds : sizes) {
        if (vg) {
            hipFuncSetAttribute((const void*)probe<1>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            hipLaunchKernelGGL(probe<1>, dim3(nwg), dim3(threads), lds, 0, d, 4000);
        } else {
            hipFuncSetAttribute((const void*)probe<0>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            hipLaunchKernelGGL(probe<0>, dim3(nwg), dim3(threads), lds, 0, d, 4000);
        }
        hipDeviceSynchronize();
        hipMemcpy(h.data(), d, sizeof(long long) * 4 * nwg, hipMemcpyDeviceToHost);
        std::map<long long, std::vector<std::pair<long long, int>>> ev;
        for (int i = 0; i < nwg; ++i) {
            long long hw = h[i * 4 + 2], xcc = h[i * 4 + 3];
            long long cu = (xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15);
            ev[cu].push_back({h[i * 4 + 0], +1});
            ev[cu].push_back({h[i * 4 + 1], -1});
        }
        int best = 0;
        for (auto& kv : ev) {
            auto v = kv.second;
            std::sort(v.begin(), v.end(), [](auto a, auto b) { return a.first < b.first || (a.first == b.first && a.second < b.second); });
            int cur = 0;
            for (auto& e : v) { cur += e.second; best = std::max(best, cur); }
        }
        printf("LDS %6d B per workgroup: max %d workgroups resident on one CU (%zu CUs seen)\n", lds,
               best, ev.size());
    }
    return 0;
}

// Internal helpers shared by the HIP translation units of libafm.so.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>

// Issue priority of the latency-bound tail kernels (rebalance, turnover / PnL scan, analyzer, FM
// solve) that run beside the FM Grams' MFMA and producer waves: at equal priority the older waves
// win every arbitration on a shared SIMD (MI355X_MICROARCH.md, two waves per SIMD).
#ifndef AFM_TAIL_PRIO
#define AFM_TAIL_PRIO 3
#endif
#ifndef AFM_SCAN_PRIO                  // the serial PnL scan and its turnover records
#define AFM_SCAN_PRIO 3
#endif
#define AFM_TAIL_PRIO_SET()                                                   \
    do {                                                                      \
        if (AFM_TAIL_PRIO) __builtin_amdgcn_s_setprio(AFM_TAIL_PRIO);         \
    } while (0)
#define AFM_SCAN_PRIO_SET()                                                   \
    do {                                                                      \
        if (AFM_SCAN_PRIO) __builtin_amdgcn_s_setprio(AFM_SCAN_PRIO);         \
    } while (0)

#include "afm.h"

struct afm_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int magic = 0x61666d31;  // "afm1"
    // execution options (afm_ctx_set_option): work splits that must not change any result, set
    // by the invariance tests; 0 = the library's choice
    int factor_split = 0;    // workgroups per 64-asset block of the factor kernel (1, 3, 5, 15)
    int factor_pair = 1;     // 3-way split: two items per workgroup
    int factor_fast = 1;     // clean-window fast step on
    int gram_checked = 0;    // afm_xs_gram_f64: checked staging only (no FAST + REDO passes)
    // factor slab calls: the work split each state buffer's layout was written with (the state
    // is [block][split][wave]; a later slab under another factor_split would misread it), and
    // the lock guarding it (host threads may share a context)
    std::unordered_map<const void*, int> slab_types;
    std::mutex slab_mu;
    // compute units of the device (hipDeviceAttributeMultiprocessorCount), read once by
    // afm_ctx_create: launch shapes that fill the chip are chosen from it
    int ncu = 256;
    // scratch buffers of the entry points, one per (slot, stream), kept across calls
    // (afm_ctx_scratch); freed by afm_ctx_destroy
    std::map<std::pair<int, hipStream_t>, std::pair<void*, size_t>> scratch;
    std::mutex scratch_mu;
};

// Scratch of an entry point: slot `slot` of the context on its current stream, at least `bytes`.
// Reused call after call in stream order (the work of one stream runs in order, so a call's
// kernels never overlap the previous call's on the same buffer); it grows only when a call needs
// more (the stream is drained first, then a new buffer).  Round 6: the per-call
// hipMallocAsync / hipFreeAsync pairs it replaces BLOCKED the host (measured with
// tools/host_probe.py on MI355X: 13.7 ms inside afm_pnl_scan_f64 and 6.2 ms inside
// afm_factors_f64 per 31-ms step), which serialised the host with the GPU every step.
enum afm_scratch_slot {
    AFM_SCRATCH_FACTOR_PARTS = 0,   // factor kernel mask partials (afm_factors_f64 / slab calls)
    AFM_SCRATCH_PNL = 1,            // afm_pnl_scan_f64 turnover records
    AFM_SCRATCH_BOOT = 2,           // afm_bootstrap_pnl_f64 path records
    AFM_SCRATCH_REB_HIST = 3,       // afm_rebalance_f64 member-major history (books > 32)
    AFM_SCRATCH_REB_SCR = 4,        // afm_rebalance_f64 window staging
    AFM_SCRATCH_POOL = 5,           // pooled-moment tree levels (xsreg.hip)
};
void* afm_ctx_scratch(afm_ctx* ctx, int slot, size_t bytes, hipError_t* err);

// the context device's compute-unit count (read when the context was created)
int afm_ctx_cus(afm_ctx* ctx);

void afm_set_error(const std::string& msg);

// Opt a kernel in to `bytes` of dynamic LDS on the context's device (> 64 KB needs it).  The
// attribute is per device, so the memo is keyed by (kernel, device): a process that drives
// several GPUs sets it on each.
hipError_t afm_lds_opt_in(const afm_ctx* ctx, const void* kernel, int bytes);

#define AFM_CHECK_ARG(cond, msg)                                   \
    do {                                                           \
        if (!(cond)) {                                             \
            afm_set_error(std::string(__func__) + ": " + (msg));   \
            return AFM_E_ARG;                                      \
        }                                                          \
    } while (0)

#define AFM_HIP(expr)                                                                     \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess) {                                                           \
            afm_set_error(std::string(__func__) + ": " #expr ": " + hipGetErrorString(_e)); \
            return AFM_E_HIP;                                                             \
        }                                                                                 \
    } while (0)

// Every entry point runs on its context's device and hands the calling thread's current device
// back on every exit path (torch and other callers rely on it): AFM_CTX validates the context and
// declares this guard in the entry point's scope.
struct afm_device_guard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit afm_device_guard(int device) {
        err = hipGetDevice(&prev);
        if (err == hipSuccess && prev != device) err = hipSetDevice(device);
        else prev = -1;                                 // already current: nothing to restore
    }
    ~afm_device_guard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    afm_device_guard(const afm_device_guard&) = delete;
    afm_device_guard& operator=(const afm_device_guard&) = delete;
};

#define AFM_CTX(ctx)                                                                      \
    if (!(ctx) || (ctx)->magic != 0x61666d31) {                                           \
        afm_set_error(std::string(__func__) + ": invalid afm_ctx");                      \
        return AFM_E_STATE;                                                               \
    }                                                                                     \
    const afm_device_guard afm_dev_guard_((ctx)->device);                                 \
    if (afm_dev_guard_.err != hipSuccess) {                                               \
        afm_set_error(std::string(__func__) + ": hipSetDevice: " +                        \
                      hipGetErrorString(afm_dev_guard_.err));                             \
        return AFM_E_HIP;                                                                 \
    }

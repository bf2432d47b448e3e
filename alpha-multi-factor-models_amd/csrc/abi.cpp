// Context, error and metadata entry points of the C-ABI (include/afm.h).
#include "afm_internal.h"

#include <map>
#include <mutex>
#include <utility>

static thread_local std::string g_last_error;

void afm_set_error(const std::string& msg) { g_last_error = msg; }

hipError_t afm_lds_opt_in(const afm_ctx* ctx, const void* kernel, int bytes) {
    static std::mutex mu;
    static std::map<std::pair<const void*, int>, int> done;    // (kernel, device) -> bytes set
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_pair(kernel, ctx->device);
    auto it = done.find(key);
    if (it != done.end() && it->second >= bytes) return hipSuccess;
    hipError_t e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done[key] = bytes;
    return e;
}

int afm_ctx_cus(afm_ctx* ctx) { return ctx->ncu; }

void* afm_ctx_scratch(afm_ctx* ctx, int slot, size_t bytes, hipError_t* err) {
    *err = hipSuccess;
    if (bytes == 0) bytes = 1;
    std::lock_guard<std::mutex> lk(ctx->scratch_mu);
    auto& e = ctx->scratch[std::make_pair(slot, ctx->stream)];
    if (e.first && e.second >= bytes) return e.first;
    if (e.first) {                       // the stream's earlier calls may still use it
        if ((*err = hipStreamSynchronize(ctx->stream)) != hipSuccess) return nullptr;
        if ((*err = hipFree(e.first)) != hipSuccess) return nullptr;
        e.first = nullptr;
        e.second = 0;
    }
    const size_t want = bytes + bytes / 4;   // headroom: a slightly larger call reuses it
    void* p = nullptr;
    if ((*err = hipMalloc(&p, want)) != hipSuccess) return nullptr;
    e.first = p;
    e.second = want;
    return p;
}

extern "C" {

const char* afm_last_error(void) { return g_last_error.c_str(); }

int afm_version(void) { return 1; }

int afm_ctx_create(int device, afm_ctx** out) {
    AFM_CHECK_ARG(out != nullptr, "out is null");
    int n = 0;
    AFM_HIP(hipGetDeviceCount(&n));
    AFM_CHECK_ARG(device >= 0 && device < n, "device ordinal out of range");
    // the CU count is read once here (no lazy init shared between host threads), and the
    // caller's current device is left as it was
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
        ncu <= 0)
        ncu = 256;                                              // MI355X
    afm_ctx* c = new afm_ctx();
    c->device = device;
    c->ncu = ncu;
    *out = c;
    return AFM_OK;
}

int afm_ctx_set_stream(afm_ctx* ctx, void* stream) {
    AFM_CTX(ctx);
    ctx->stream = reinterpret_cast<hipStream_t>(stream);
    return AFM_OK;
}

int afm_ctx_set_option(afm_ctx* ctx, const char* name, int64_t value) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(name != nullptr, "name is null");
    const std::string n(name);
    if (n == "factor_split") {
        AFM_CHECK_ARG(value == 0 || value == 1 || value == 3 || value == 5 || value == 15 ||
                          value == 103 || value == 105 || value == 106 || value == 110 ||
                          value == 206,
                      "factor_split: 0 (auto); 1, 3, 5 or 15 (the 15-set partition); 103, 105, "
                      "106 or 110 (the 30-set small-grid partition); 206 (the 60-set "
                      "partition)");
        ctx->factor_split = (int)value;
    } else if (n == "factor_pair") {
        ctx->factor_pair = value != 0;
    } else if (n == "factor_fast") {
        ctx->factor_fast = value != 0;
    } else if (n == "gram_checked") {
        ctx->gram_checked = value != 0;
    } else {
        AFM_CHECK_ARG(false, "unknown option " + n);
    }
    return AFM_OK;
}

int afm_ctx_get_option(afm_ctx* ctx, const char* name, int64_t* value) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(name != nullptr && value != nullptr, "null argument");
    const std::string n(name);
    if (n == "factor_split") *value = ctx->factor_split;
    else if (n == "factor_pair") *value = ctx->factor_pair ? 1 : 0;
    else if (n == "factor_fast") *value = ctx->factor_fast ? 1 : 0;
    else if (n == "gram_checked") *value = ctx->gram_checked ? 1 : 0;
    else AFM_CHECK_ARG(false, "unknown option " + n);
    return AFM_OK;
}

int afm_stream_create_cu_mask(int device, const uint32_t* cu_mask, int nwords, void** out) {
    AFM_CHECK_ARG(out != nullptr && cu_mask != nullptr && nwords > 0, "null argument");
    int n = 0;
    AFM_HIP(hipGetDeviceCount(&n));
    AFM_CHECK_ARG(device >= 0 && device < n, "device ordinal out of range");
    // the stream belongs to `device`; the calling thread's current device is restored on every
    // exit path (torch and other callers rely on it)
    int prev = 0;
    AFM_HIP(hipGetDevice(&prev));
    AFM_HIP(hipSetDevice(device));
    hipStream_t s = nullptr;
    const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, cu_mask);
    const hipError_t r = hipSetDevice(prev);
    AFM_HIP(e);
    AFM_HIP(r);
    *out = (void*)s;
    return AFM_OK;
}

int afm_stream_destroy(void* stream) {
    AFM_CHECK_ARG(stream != nullptr, "null stream");
    AFM_HIP(hipStreamDestroy(reinterpret_cast<hipStream_t>(stream)));
    return AFM_OK;
}

int afm_ctx_destroy(afm_ctx* ctx) {
    if (!ctx || ctx->magic != 0x61666d31) {
        afm_set_error("afm_ctx_destroy: invalid afm_ctx");
        return AFM_E_STATE;
    }
    ctx->magic = 0;
    if (!ctx->scratch.empty()) {
        const afm_device_guard dg(ctx->device);
        (void)hipDeviceSynchronize();
        for (auto& kv : ctx->scratch)
            if (kv.second.first) (void)hipFree(kv.second.first);
    }
    delete ctx;
    return AFM_OK;
}

static const char* kFactorNames[AFM_N_FACTORS] = {
    "SMA_6", "SMA_10", "SMA_14", "SMA_18", "SMA_22", "SMA_26", "SMA_30", "SMA_34", "SMA_38",
    "SMA_42", "SMA_46", "SMA_50",
    "EMA_6", "EMA_10", "EMA_14", "EMA_18", "EMA_22", "EMA_26", "EMA_30", "EMA_34", "EMA_38",
    "EMA_42", "EMA_46", "EMA_50",
    "VWMA_6", "VWMA_10", "VWMA_14", "VWMA_18", "VWMA_22", "VWMA_26", "VWMA_30", "VWMA_34",
    "VWMA_38", "VWMA_42", "VWMA_46", "VWMA_50",
    "BBANDS_upper_14", "BBANDS_lower_14", "BBANDS_upper_20", "BBANDS_lower_20",
    "BBANDS_upper_26", "BBANDS_lower_26", "BBANDS_upper_32", "BBANDS_lower_32",
    "BBANDS_upper_38", "BBANDS_lower_38", "BBANDS_upper_44", "BBANDS_lower_44",
    "BBANDS_upper_50", "BBANDS_lower_50", "BBANDS_upper_56", "BBANDS_lower_56",
    "MOM_14", "MOM_20", "MOM_26", "MOM_32", "MOM_38", "MOM_44", "MOM_50", "MOM_56",
    "ACCEL_14", "ACCEL_20", "ACCEL_26", "ACCEL_32", "ACCEL_38", "ACCEL_44", "ACCEL_50", "ACCEL_56",
    "ROCR_14", "ROCR_20", "ROCR_26", "ROCR_32", "ROCR_38", "ROCR_44", "ROCR_50", "ROCR_56",
    "MACD_12_18", "MACD_12_24", "MACD_12_30",
    "RSI_8", "RSI_14", "RSI_20",
    "PVT", "OBV", "PSY",
    "sd_3", "sd_5", "sd_15", "sd5_15",
    "volsd_3", "volsd_5", "volsd_15", "volsd5_15",
    "vol_change", "corr_5", "corr_15",
    "target", "tmr_ret1d",
};

const char* afm_factor_name(int i) {
    if (i < 0 || i >= AFM_N_FACTORS) return nullptr;
    return kFactorNames[i];
}

}  // extern "C"

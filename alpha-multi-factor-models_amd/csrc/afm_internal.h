// Internal helpers shared by the HIP translation units of libafm.so.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "afm.h"

struct afm_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int magic = 0x61666d31;  // "afm1"
};

void afm_set_error(const std::string& msg);

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

#define AFM_CTX(ctx)                                                      \
    do {                                                                  \
        if (!(ctx) || (ctx)->magic != 0x61666d31) {                       \
            afm_set_error(std::string(__func__) + ": invalid afm_ctx");  \
            return AFM_E_STATE;                                           \
        }                                                                 \
        AFM_HIP(hipSetDevice((ctx)->device));                             \
    } while (0)

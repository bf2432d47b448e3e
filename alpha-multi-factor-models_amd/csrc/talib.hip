// talib factor variant: the TA-Lib columns of the reference's second
// compute_factors (KKT Yuliang Jiang.py:176-270).  The columns it shares with No-talib.py (MOM,
// ACCEL, ROCR, PSY, sd, volsd, vol_change, corr, target, tmr_ret1d) are pandas-exact and come from
// factors.hip; this kernel computes the 68 that TA-Lib defines differently:
//   SMA_i, EMA_i, VSMA_i (i = 6..50 step 4), BBANDS upper/middle/lower (i = 14..56 step 6),
//   MACD_12_i (i = 18, 24, 30; signal 9), RSI_i (i = 8, 14, 20), PVT (no cumsum), OBV (TA-Lib).
// TA-Lib is not installed here, so the semantics are restated from TA-Lib 0.4 C core
// (TA_COMPATIBILITY_DEFAULT, unstable periods 0): ta_SMA.c TA_INT_SMA (running total: add the new
// value, emit total / n, subtract the oldest), ta_EMA.c TA_INT_EMA (seed = sequential sum of the
// first n values / n at index n - 1, then prev = (x - prev) * k + prev, k = 2 / (n + 1)),
// ta_BBANDS.c with TA_INT_stddev_using_precalc_ma (running sum of squares, var = total2 / n -
// middle^2, 0 when var < 1e-8, bands = middle +- 2 * sd), ta_MACD.c TA_INT_MACD (fast and slow
// EMAs both started at index slow - 1 -- the fast one seeded with the mean of the 12 values ending
// there -- output from index slow - 1 + 8, the signal EMA's lookback), ta_RSI.c (Wilder: mean
// gain / loss of the first n differences, then (prev * (n - 1) + x) / n; 0 when |gain + loss| <
// 1e-8), ta_OBV.c (starts at volume[0]; equal closes leave it unchanged).  Parity: bit-exact with
// the C restatement oracle/talib_oracle.c; against TA-Lib itself parity is UNPINNED (no TA-Lib,
// no TA-Lib outputs in the reference).
//
// Four waves per 64-asset block (lane = asset), each owning a column group and walking the
// asset's present days sequentially: windows are positional over observations (one DataFrame
// per security, KKT:183-185).  64-slot LDS rings per lane hold the last close (and volume *
// close) values for the windowed groups.
#include "afm_internal.h"

#pragma clang fp contract(off)

namespace afm {
namespace {

constexpr int kTlRing = 64;
constexpr int kTlCols = 68;

__device__ __forceinline__ double tnan() { return __builtin_nan(""); }

struct TlArgs {
    int64_t T, lda, plane;
    const double* close;
    const double* volume;
    const uint64_t* vbits;
    double* out;              // [68][T][lda]
};

// Role r of a block's four waves (lane = asset; each wave walks the presence words itself):
//   0: SMA + VSMA (close and volume*close rings)   1: EMA + MACD
//   2: BBANDS (close ring)                          3: RSI, PVT, OBV
template <int ROLE>
__device__ void talib_wave(const TlArgs& a, double (*rc)[64], double (*rv)[64], int lane,
                           int64_t asset) {
    double s0[12], s1[12];                           // role 0: SMA / VSMA totals; 1: EMA
    double b0[8], b1[8];                             // role 2: BBANDS totals
    double m0[3], m1[3], m2[3];                      // role 1: MACD slow / fast / fast seed;
                                                     // role 3: RSI gain / loss
    for (int j = 0; j < 12; ++j) { s0[j] = 0.0; s1[j] = 0.0; }
    for (int j = 0; j < 8; ++j) { b0[j] = 0.0; b1[j] = 0.0; }
    for (int j = 0; j < 3; ++j) { m0[j] = 0.0; m1[j] = 0.0; m2[j] = 0.0; }
    double obv = 0.0, prevc = 0.0;
    int p = 0;                                       // observations so far
    const int64_t nch = (a.T + 63) / 64;
    for (int64_t ch = 0; ch < nch; ++ch) {
        uint64_t w = a.vbits[ch * a.lda + asset];
        while (w) {
            const int64_t t = ch * 64 + __builtin_ctzll(w);
            w &= w - 1;
            const int64_t cell = t * a.lda + asset;
            const double c = a.close[cell], v = a.volume[cell];
            double* o = a.out + cell;
            if (ROLE == 0) {                         // SMA / VSMA (TA_INT_SMA)
                const double vc = v * c;
                rc[p & 63][lane] = c;
                rv[p & 63][lane] = vc;
                for (int j = 0; j < 12; ++j) {
                    const int n = 6 + 4 * j;
                    s0[j] = s0[j] + c;
                    s1[j] = s1[j] + vc;
                    double sm = tnan(), vs = tnan();
                    if (p >= n - 1) {
                        sm = s0[j] / (double)n;
                        vs = s1[j] / (double)n;
                        s0[j] = s0[j] - rc[(p - n + 1) & 63][lane];
                        s1[j] = s1[j] - rv[(p - n + 1) & 63][lane];
                    }
                    o[(int64_t)j * a.plane] = sm;
                    o[(int64_t)(24 + j) * a.plane] = vs;
                }
            } else if (ROLE == 1) {                  // EMA (TA_INT_EMA), MACD (TA_INT_MACD)
                for (int j = 0; j < 12; ++j) {
                    const int n = 6 + 4 * j;
                    double e = tnan();
                    if (p < n - 1) {
                        s0[j] = s0[j] + c;           // sequential seed sum
                    } else if (p == n - 1) {
                        s0[j] = (s0[j] + c) / (double)n;
                        e = s0[j];
                    } else {
                        s0[j] = ((c - s0[j]) * (2.0 / (double)(n + 1))) + s0[j];
                        e = s0[j];
                    }
                    o[(int64_t)(12 + j) * a.plane] = e;
                }
                for (int j = 0; j < 3; ++j) {        // both EMAs start at index slow - 1
                    const int sl = 18 + 6 * j;
                    double m = tnan();
                    if (p < sl - 1) {
                        m0[j] = m0[j] + c;
                        if (p >= sl - 12) m2[j] = m2[j] + c;
                    } else if (p == sl - 1) {
                        m0[j] = (m0[j] + c) / (double)sl;
                        m1[j] = (m2[j] + c) / 12.0;
                    } else {
                        m1[j] = ((c - m1[j]) * (2.0 / 13.0)) + m1[j];
                        m0[j] = ((c - m0[j]) * (2.0 / (double)(sl + 1))) + m0[j];
                    }
                    if (p >= sl - 1 + 8) m = m1[j] - m0[j];
                    o[(int64_t)(60 + j) * a.plane] = m;
                }
            } else if (ROLE == 2) {                  // BBANDS (SMA middle, precalc-MA stddev)
                rc[p & 63][lane] = c;
                for (int j = 0; j < 8; ++j) {
                    const int n = 14 + 6 * j;
                    b0[j] = b0[j] + c;
                    b1[j] = b1[j] + c * c;
                    double up = tnan(), mid = tnan(), lo = tnan();
                    if (p >= n - 1) {
                        mid = b0[j] / (double)n;
                        double mv2 = b1[j] / (double)n;
                        const double old = rc[(p - n + 1) & 63][lane];
                        b0[j] = b0[j] - old;
                        b1[j] = b1[j] - old * old;
                        mv2 = mv2 - mid * mid;
                        const double sd = (mv2 < 0.00000001) ? 0.0 : __builtin_sqrt(mv2);
                        const double d = sd * 2.0;
                        up = mid + d;
                        lo = mid - d;
                    }
                    o[(int64_t)(36 + 3 * j) * a.plane] = up;
                    o[(int64_t)(37 + 3 * j) * a.plane] = mid;
                    o[(int64_t)(38 + 3 * j) * a.plane] = lo;
                }
            } else {                                 // RSI (Wilder), PVT, OBV
                const double d = c - prevc;
                for (int j = 0; j < 3; ++j) {
                    const int n = 8 + 6 * j;
                    double r = tnan();
                    if (p >= 1 && p <= n) {
                        if (d < 0) m1[j] = m1[j] - d; else m0[j] = m0[j] + d;
                        if (p == n) {
                            m1[j] = m1[j] / (double)n;
                            m0[j] = m0[j] / (double)n;
                        }
                    } else if (p > n) {
                        m1[j] = m1[j] * (double)(n - 1);
                        m0[j] = m0[j] * (double)(n - 1);
                        if (d < 0) m1[j] = m1[j] - d; else m0[j] = m0[j] + d;
                        m1[j] = m1[j] / (double)n;
                        m0[j] = m0[j] / (double)n;
                    }
                    if (p >= n) {
                        const double sg = m0[j] + m1[j];
                        r = (-0.00000001 < sg && sg < 0.00000001) ? 0.0 : 100.0 * (m0[j] / sg);
                    }
                    o[(int64_t)(63 + j) * a.plane] = r;
                }
                if (p == 0) obv = v;
                else if (c > prevc) obv = obv + v;
                else if (c < prevc) obv = obv - v;
                o[(int64_t)66 * a.plane] = p >= 1 ? v * (c / prevc - 1) : tnan();
                o[(int64_t)67 * a.plane] = obv;
            }
            prevc = c;
            ++p;
        }
    }
}

__global__ __launch_bounds__(256) void talib_kernel(TlArgs a) {
    __shared__ double rc0[kTlRing][64], rv0[kTlRing][64], rc2[kTlRing][64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t asset = (int64_t)blockIdx.x * 64 + lane;
    switch (wave) {
        case 0: talib_wave<0>(a, rc0, rv0, lane, asset); break;
        case 1: talib_wave<1>(a, nullptr, nullptr, lane, asset); break;
        case 2: talib_wave<2>(a, rc2, nullptr, lane, asset); break;
        default: talib_wave<3>(a, nullptr, nullptr, lane, asset); break;
    }
}

}  // namespace
}  // namespace afm

extern "C" int afm_talib_factors_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda,
                                     const double* close, const double* volume,
                                     const uint64_t* valid_bits, double* out) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(T > 0 && A > 0, "T and A must be positive");
    AFM_CHECK_ARG(lda >= A && lda % 64 == 0, "lda must be a multiple of 64 and >= A");
    AFM_CHECK_ARG(close && volume && valid_bits && out, "null buffer");
    afm::TlArgs g{T, lda, T * lda, close, volume, valid_bits, out};
    hipLaunchKernelGGL(afm::talib_kernel, dim3((unsigned)((A + 63) / 64)), dim3(256), 0,
                       ctx->stream, g);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

// Per-security z-score of the feature columns (KKT Yuliang Jiang.py:446-458):
//   sigma = df_train_x.groupby('security_id').std(); mu = ....mean()           (KKT:446-447)
//   df_*_x = ((x - mu) / sigma).replace([inf, -inf], nan).dropna()            (KKT:449-451)
//
// Two HBM passes over calendar-grid planes [T][lda] (lanes = consecutive assets of one date, so
// every access is a coalesced 512-B row segment):
//   zscore_stats_kernel  one thread per (column, asset): a sequential scan over the train dates
//                        with pandas' group_mean (Kahan, NaN compensation reset) and group_var
//                        (Welford, ddof = 1) recurrences, in the same row order as the groupby
//                        (ascending date within a security).  Reads 8 B per (column, train row).
//   zscore_apply_kernel  one thread per (asset, 64-day chunk): z = (x - mu) / sigma with IEEE
//                        subtract and divide (no reciprocal: bit-exact with pandas), +-inf -> NaN,
//                        and the dropna() row bits = rows with every column non-NaN.
//                        Reads 8 B and writes 8 B per (column, row).
// Both are HBM-bound (SURVEY §8(d) "cheap HBM pass"): algorithmic bytes per (column, row) are 8
// (stats, train rows) and 16 (apply, applied rows).
#include "afm_internal.h"

#pragma clang fp contract(off)

namespace afm {
namespace {

typedef unsigned long long u64;

constexpr int kUnroll = 8;
constexpr int64_t kStatsTabMax = 48 * 1024;   // reciprocal table bytes (6,143 train dates)

__device__ __forceinline__ double qnan() { return __builtin_nan(""); }

// grid (ceil(lda / NT), K); thread = (column k = blockIdx.y, asset a).
// TAB: the Welford quotient (val - old) / nobs by Markstein's correction from the correctly
// rounded reciprocal RN(1 / nobs), read from an LDS table the workgroup fills first (t1 - t0 + 1
// entries): q0 = x r, e = fma(-q0, n, x), q = fma(e, r, q0) is the IEEE quotient when nothing
// under- or overflows (the same identity as lasso.hip div_r / analyzer.hip; a quotient outside
// [2^-400, 2^400], a zero, an infinity or a NaN takes the IEEE division).  That is 3 f64
// operations for the ~11 of the division sequence, with the count kept as a double (no
// int64 -> f64 conversion per row).  1024 threads so the table is shared by 16 waves (256 when
// the grid is too small to fill the chip that way).
template <int NT, bool TAB>
__global__ __launch_bounds__(NT) void zscore_stats_kernel(const double* base, int64_t col_stride,
                                                          int64_t lda, const int32_t* cols,
                                                          const uint64_t* bits, int64_t t0,
                                                          int64_t t1, double* mu, double* sd) {
    extern __shared__ double rtab[];                    // [t1 - t0 + 1]: RN(1 / n), TAB only
    if (TAB) {
        for (int i = threadIdx.x; i <= (int)(t1 - t0); i += NT) rtab[i] = 1.0 / (double)i;
        __syncthreads();
    }
    const int64_t a = (int64_t)blockIdx.x * NT + threadIdx.x;
    const int k = blockIdx.y;
    if (a >= lda) return;
    const double* x = base + (int64_t)cols[k] * col_stride + a;
    // group_mean: Kahan sum with the compensation reset when it turns NaN
    double sum = 0.0, comp = 0.0;
    // group_var: Welford
    double mean = 0.0, m2 = 0.0;
    int nobs = 0;                                       // (dates < 2^31)
    double dn = 0.0;                                    // nobs as a double (exact below 2^53)
    for (int64_t c = t0 >> 6; c <= (t1 - 1) >> 6; ++c) {
        u64 w = bits[c * lda + a];
        const int64_t d0 = c << 6;
        if (d0 < t0) w &= ~0ull << (t0 - d0);
        if (t1 - d0 < 64) w &= (1ull << (t1 - d0)) - 1ull;
        // days of this chunk in blocks of kUnroll: the loads of a block are issued together
        for (int j0 = 0; j0 < 64; j0 += kUnroll) {
            const u64 wb = (w >> j0) & ((1ull << kUnroll) - 1ull);
            if (!__any(wb != 0)) continue;
            double v[kUnroll];
#pragma unroll
            for (int j = 0; j < kUnroll; ++j)
                v[j] = ((wb >> j) & 1ull) ? x[(d0 + j0 + j) * lda] : qnan();
#pragma unroll
            for (int j = 0; j < kUnroll; ++j) {
                const double val = v[j];
                if (val == val) {                       // absent rows read NaN: skipped
                    nobs += 1;
                    const double y = val - comp;
                    const double t = sum + y;
                    comp = t - sum - y;
                    if (comp != comp) comp = 0.0;
                    sum = t;
                    const double old = mean;
                    if (TAB) {
                        dn = dn + 1.0;
                        const double dx = val - old, r = rtab[nobs];
                        const double q0 = dx * r;
                        const double e = __builtin_fma(-q0, dn, dx);
                        double q = __builtin_fma(e, r, q0);
                        const double aq = __builtin_fabs(q0);
                        if (!(aq > 0x1p-400 && aq < 0x1p400)) {
                            double xd = dx;             // (volatile: the division stays behind
                            asm volatile("" : "+v"(xd));   // the branch, not speculated)
                            q = xd / dn;
                        }
                        mean = mean + q;
                    } else {
                        mean = mean + (val - old) / (double)nobs;
                    }
                    m2 = m2 + (val - mean) * (val - old);
                }
            }
        }
    }
    const double ct = (double)nobs;
    mu[(int64_t)k * lda + a] = nobs == 0 ? qnan() : sum / ct;
    sd[(int64_t)k * lda + a] = nobs <= 1 ? qnan() : __builtin_sqrt(m2 / (ct - 1.0));
}

// Streamed z statistics (round 5; the smallest grids, beside the factor kernel's time slabs): the
// same recurrences over the dates [t0, t1) of one slab, each (column, asset) state -- Kahan sum and
// compensation, Welford mean and M2, the count -- carried in st [5][K][lda] between slabs (first:
// start from zero; last: write mu / sd, else store the state).  The Welford quotient is the IEEE
// division (the value the reciprocal table's Markstein step reproduces), so the kernel needs no
// LDS and its waves fit beside a factor workgroup that holds 140 KB of a CU.  Bitwise the
// statistics of one zscore_stats_kernel pass over the union of the slabs.
__global__ __launch_bounds__(256) void zscore_stats_slab_kernel(const double* base,
                                                                int64_t col_stride, int64_t lda,
                                                                const int32_t* cols, int K,
                                                                const uint64_t* bits, int64_t t0,
                                                                int64_t t1, double* st, int first,
                                                                int last, double* mu, double* sd) {
    const int64_t a = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int k = blockIdx.y;
    if (a >= lda) return;
    const double* x = base + (int64_t)cols[k] * col_stride + a;
    const int64_t sl = (int64_t)K * lda, si = (int64_t)k * lda + a;
    double sum = 0.0, comp = 0.0, mean = 0.0, m2 = 0.0;
    int nobs = 0;
    if (!first) {
        sum = st[si];
        comp = st[sl + si];
        mean = st[2 * sl + si];
        m2 = st[3 * sl + si];
        nobs = (int)st[4 * sl + si];
    }
    for (int64_t c = t0 >> 6; c <= (t1 - 1) >> 6; ++c) {
        u64 w = bits[c * lda + a];
        const int64_t d0 = c << 6;
        if (d0 < t0) w &= ~0ull << (t0 - d0);
        if (t1 - d0 < 64) w &= (1ull << (t1 - d0)) - 1ull;
        for (int j0 = 0; j0 < 64; j0 += kUnroll) {
            const u64 wb = (w >> j0) & ((1ull << kUnroll) - 1ull);
            if (!__any(wb != 0)) continue;
            double v[kUnroll];
#pragma unroll
            for (int j = 0; j < kUnroll; ++j)
                v[j] = ((wb >> j) & 1ull) ? x[(d0 + j0 + j) * lda] : qnan();
#pragma unroll
            for (int j = 0; j < kUnroll; ++j) {
                const double val = v[j];
                if (val == val) {                       // absent rows read NaN: skipped
                    nobs += 1;
                    const double y = val - comp;
                    const double t = sum + y;
                    comp = t - sum - y;
                    if (comp != comp) comp = 0.0;
                    sum = t;
                    const double old = mean;
                    mean = mean + (val - old) / (double)nobs;
                    m2 = m2 + (val - mean) * (val - old);
                }
            }
        }
    }
    if (last) {
        const double ct = (double)nobs;
        mu[si] = nobs == 0 ? qnan() : sum / ct;
        sd[si] = nobs <= 1 ? qnan() : __builtin_sqrt(m2 / (ct - 1.0));
    } else {
        st[si] = sum;
        st[sl + si] = comp;
        st[2 * sl + si] = mean;
        st[3 * sl + si] = m2;
        st[4 * sl + si] = (double)nobs;
    }
}

// grid (ceil(lda / 256), chunks of [t0, t1)); thread = (asset a, chunk c)
__global__ __launch_bounds__(256) void zscore_apply_kernel(const double* base, int64_t col_stride,
                                                           int64_t lda, const int32_t* cols, int K,
                                                           const uint64_t* bits, int64_t t0,
                                                           int64_t t1, const double* mu,
                                                           const double* sd, double* out,
                                                           int64_t out_col_stride,
                                                           const int32_t* out_cols,
                                                           uint64_t* keep) {
    const int64_t a = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t c = (t0 >> 6) + blockIdx.y;
    if (a >= lda) return;
    u64 w = bits[c * lda + a];
    const int64_t d0 = c << 6;
    if (d0 < t0) w &= ~0ull << (t0 - d0);
    if (t1 - d0 < 64) w &= (1ull << (t1 - d0)) - 1ull;
    u64 bad = 0;
    if (__any(w != 0)) {
        const int64_t cell = d0 * lda + a;
        for (int k = 0; k < K; ++k) {
            const double m = mu[(int64_t)k * lda + a], s = sd[(int64_t)k * lda + a];
            const double* x = base + (int64_t)cols[k] * col_stride + cell;
            double* o = out + (int64_t)out_cols[k] * out_col_stride + cell;
            for (int j0 = 0; j0 < 64; j0 += kUnroll) {
                const u64 wb = (w >> j0) & ((1ull << kUnroll) - 1ull);
                if (!__any(wb != 0)) continue;
                double v[kUnroll];
#pragma unroll
                for (int j = 0; j < kUnroll; ++j)
                    v[j] = ((wb >> j) & 1ull) ? x[(j0 + j) * lda] : 0.0;
#pragma unroll
                for (int j = 0; j < kUnroll; ++j) {
                    if ((wb >> j) & 1ull) {
                        double z = (v[j] - m) / s;
                        if (__builtin_isinf(z)) z = qnan();
                        bad |= (u64)(z != z) << (j0 + j);
                        o[(j0 + j) * lda] = z;
                    }
                }
            }
        }
    }
    keep[c * lda + a] = w & ~bad;
}

}  // namespace
}  // namespace afm

using namespace afm;

extern "C" int afm_zscore_stats_f64(afm_ctx* ctx, const double* base, int64_t col_stride,
                                    int64_t T, int64_t lda, const int32_t* cols, int K,
                                    const uint64_t* bits, int64_t t0, int64_t t1, double* mu,
                                    double* sd) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(base && cols && bits && mu && sd, "null buffer");
    AFM_CHECK_ARG(lda > 0 && lda % 64 == 0 && K >= 1 && K <= 65535, "bad shape");
    AFM_CHECK_ARG(col_stride >= T * lda, "col_stride smaller than a [T][lda] plane");
    AFM_CHECK_ARG(0 <= t0 && t0 <= t1 && t1 <= T, "bad date range");
    if (t0 == t1) {
        AFM_HIP(hipMemsetAsync(mu, 0xff, sizeof(double) * K * lda, ctx->stream));   // NaN
        AFM_HIP(hipMemsetAsync(sd, 0xff, sizeof(double) * K * lda, ctx->stream));
        return AFM_OK;
    }
    const int64_t tab = (t1 - t0 + 1) * (int64_t)sizeof(double);
    // 1,024-thread workgroups (one table per 16 waves) when they fill the chip at two per CU;
    // a smaller grid (the per-rank shards) keeps 256-thread workgroups, so no CU sits idle
    const int64_t wg1024 = (lda + 1023) / 1024 * K;
    if (tab <= kStatsTabMax && wg1024 >= 2 * (int64_t)afm_ctx_cus(ctx)) {
        dim3 grid((unsigned)((lda + 1023) / 1024), (unsigned)K);
        hipLaunchKernelGGL((zscore_stats_kernel<1024, true>), grid, dim3(1024), (unsigned)tab,
                           ctx->stream, base, col_stride, lda, cols, bits, t0, t1, mu, sd);
    } else if (tab <= kStatsTabMax) {
        dim3 grid((unsigned)((lda + 255) / 256), (unsigned)K);
        hipLaunchKernelGGL((zscore_stats_kernel<256, true>), grid, dim3(256), (unsigned)tab,
                           ctx->stream, base, col_stride, lda, cols, bits, t0, t1, mu, sd);
    } else {
        dim3 grid((unsigned)((lda + 255) / 256), (unsigned)K);
        hipLaunchKernelGGL((zscore_stats_kernel<256, false>), grid, dim3(256), 0, ctx->stream,
                           base, col_stride, lda, cols, bits, t0, t1, mu, sd);
    }
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_zscore_stats_slab_f64(afm_ctx* ctx, const double* base, int64_t col_stride,
                                         int64_t T, int64_t lda, const int32_t* cols, int K,
                                         const uint64_t* bits, int64_t t0, int64_t t1,
                                         double* state, int first, int last, double* mu,
                                         double* sd) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(base && cols && bits && state && (!last || (mu && sd)), "null buffer");
    AFM_CHECK_ARG(lda > 0 && lda % 64 == 0 && K >= 1 && K <= 65535, "bad shape");
    AFM_CHECK_ARG(col_stride >= T * lda, "col_stride smaller than a [T][lda] plane");
    AFM_CHECK_ARG(0 <= t0 && t0 < t1 && t1 <= T, "bad date range (a slab holds at least one date)");
    dim3 grid((unsigned)((lda + 255) / 256), (unsigned)K);
    hipLaunchKernelGGL(zscore_stats_slab_kernel, grid, dim3(256), 0, ctx->stream, base, col_stride,
                       lda, cols, K, bits, t0, t1, state, first, last, mu, sd);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_zscore_apply_f64(afm_ctx* ctx, const double* base, int64_t col_stride,
                                    int64_t T, int64_t lda, const int32_t* cols, int K,
                                    const uint64_t* bits, int64_t t0, int64_t t1,
                                    const double* mu, const double* sd, double* out,
                                    int64_t out_col_stride, const int32_t* out_cols,
                                    uint64_t* keep) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(base && cols && bits && mu && sd && out && out_cols && keep, "null buffer");
    AFM_CHECK_ARG(lda > 0 && lda % 64 == 0 && K >= 1, "bad shape");
    AFM_CHECK_ARG(col_stride >= T * lda && out_col_stride >= T * lda,
                  "col_stride smaller than a [T][lda] plane");
    AFM_CHECK_ARG(0 <= t0 && t0 <= t1 && t1 <= T, "bad date range");
    if (t0 == t1) return AFM_OK;
    const int64_t nch = ((t1 - 1) >> 6) - (t0 >> 6) + 1;
    dim3 grid((unsigned)((lda + 255) / 256), (unsigned)nch);
    hipLaunchKernelGGL(zscore_apply_kernel, grid, dim3(256), 0, ctx->stream, base, col_stride,
                       lda, cols, K, bits, t0, t1, mu, sd, out, out_col_stride, out_cols, keep);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

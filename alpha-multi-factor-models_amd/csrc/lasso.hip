// Lasso on the pooled Gram: the reference fits
// sklearn Lasso(alpha=2e-4, max_iter=10000) on the pooled train+valid design
// (KKT Yuliang Jiang.py:605-607).  The design's centered moments already exist on the device:
// the per-segment shifted Grams (xsreg.hip gram_kernel) combined by pool_kernel.  So the fit is
// cyclic coordinate descent on the centered Gram -- sklearn's enet_coordinate_descent_gram
// (linear_model/_cd_fast.pyx, sklearn 1.7.2): H = Q w maintained by two axpys per coordinate,
// soft-threshold update, stopping rule w_max == 0 or d_w_max / w_max < tol (or the last
// iteration) followed by the duality gap test gap < tol * y'y.  Same operation order as
// oracle/lasso_oracle.c (axpy = one fma per element, reductions sequential in feature order).
//
// One wave (after a block-wide setup of Q): lane j owns features j and j + 64 (p <= 110); H, w
// and q live in registers; coordinates that cannot move are skipped by ballot (a sweep costs its
// movable coordinates, not p); the Gram
// Q sits in LDS (a row per coordinate, conflict-free); a coordinate's step runs on its half's
// registers in every lane of that half (lane c's result kept, then broadcast to the axpys).  The
// work is a few hundred flops per coordinate on one in-order wave: its instruction count and
// dependency chain bound it (one date-free solve per fit, ~microseconds per sweep).
#include "afm_internal.h"

#pragma clang fp contract(off)

namespace afm {
namespace {

constexpr int kMaxLassoP = 110;
constexpr int kQS = 128;                 // LDS row stride of Q (doubles): lanes j and j + 64

__device__ __forceinline__ double bcast(double v, int lane) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, lane);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), lane);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// value of feature j from the (v0: j < 64, v1: j >= 64) register pair, j uniform: both lanes
// read, then a scalar select (no branch on the coordinate's half)
__device__ __forceinline__ double pick(double v0, double v1, int j) {
    const double a = bcast(v0, j & 63), b = bcast(v1, j & 63);
    return j < 64 ? a : b;
}
__device__ __forceinline__ double fsign(double f) { return f == 0.0 ? 0.0 : (f > 0.0 ? 1.0 : -1.0); }
// computed here: an empty volatile asm on the value keeps the compiler from sinking its
// producer into a later branch or behind a longer chain
__device__ __forceinline__ void pin(double& v) { __asm__ volatile("" : "+v"(v)); }
// The quotient x / d with r = RN(1 / d) by Markstein's correction q0 = RN(x r), e = fma(-q0, d, x),
// q = RN(q0 + e r) is the IEEE quotient when r is the correctly rounded reciprocal and nothing
// under- or overflows (checked on 5.6e8 hard and random cases, tools/markstein_any.c).  A zero x
// gives x itself (d > 0: the signed zero the division would give); a quotient outside
// [2^-400, 2^400] takes the IEEE division (a uniform branch, never in practice).  (`solve` below.)

// alpha_row >= 0: alpha = alpha_row * n (sklearn's alpha times the row count, read on the device);
// shift / beta_out (optional): beta_out = [intercept, w] with sklearn's _set_intercept,
// intercept = y_offset - X_offset . w over the pooled means (shift + G'[0][.] / n).
constexpr int kLassoThreads = 1024;   // the setup of Q; wave 0 alone runs the descent

// POS: sklearn's positive=True (a launch-time constant: no per-coordinate branch on it)
template <bool POS>
__global__ __launch_bounds__(kLassoThreads) void lasso_cd_kernel(const double* gram, int p, double alpha,
                                                      double beta, int max_iter, double tol,
                                                      double* w_out, double* info,
                                                      double alpha_row, const double* shift,
                                                      double* beta_out) {
    extern __shared__ double Q[];                    // [p][kQS] centered X'X, zero past column p
    const int tid = threadIdx.x, lane = tid & 63;
    const int p2 = p + 2;
    const double n = gram[0];
    if (alpha_row >= 0.0) alpha = alpha_row * n;
    // centered moments C = G'[1:,1:] - (g0 g0^T) / n of [x, y] (oracle.centered_moments), by the
    // whole block: a lone wave took ~150 dependent rounds of L2 loads and a division here
    for (int e = tid; e < p * kQS; e += kLassoThreads) {
        const int i = e / kQS, j = e - i * kQS;
        Q[e] = j < p ? gram[(1 + i) * p2 + 1 + j] - (gram[1 + i] * gram[1 + j]) / n : 0.0;
    }
    __syncthreads();
    if (tid >= 64) return;
    const int j0 = lane, j1 = lane + 64;
    const bool has0 = j0 < p, has1 = j1 < p;
    double q0 = 0.0, q1 = 0.0;
    if (has0) q0 = gram[(1 + j0) * p2 + 1 + p] - (gram[1 + j0] * gram[1 + p]) / n;
    if (has1) q1 = gram[(1 + j1) * p2 + 1 + p] - (gram[1 + j1] * gram[1 + p]) / n;
    const double ynorm2 = gram[(1 + p) * p2 + 1 + p] - (gram[1 + p] * gram[1 + p]) / n;

    double h0 = 0.0, h1 = 0.0, w0 = 0.0, w1 = 0.0;  // H = Q w, w (start at 0: H = 0)
    double gap = tol + 1.0;
    const double d_w_tol = tol;
    const double tol_y = tol * ynorm2;
    int n_iter = 0;
    // per-lane diagonal: a coordinate whose weight is 0 and whose soft threshold gives 0 again
    // changes nothing (no H update, w stays a signed zero) -- the sweep skips to the next
    // coordinate that can move, found by ballot over the lanes' current H
    const double qd0 = has0 ? Q[j0 * kQS + j0] : 0.0, qd1 = has1 ? Q[j1 * kQS + j1] : 0.0;
    // the soft-threshold divisors qii + beta and their correctly rounded reciprocals (a divisor
    // whose reciprocal is not normal keeps the IEEE division: rd = 0 marks it)
    const double dd0 = qd0 + beta, dd1 = qd1 + beta;
    double rd0 = 1.0 / dd0, rd1 = 1.0 / dd1;
    if (!(__builtin_fabs(rd0) > 0x1p-400 && __builtin_fabs(rd0) < 0x1p400)) rd0 = 0.0;
    if (!(__builtin_fabs(rd1) > 0x1p-400 && __builtin_fabs(rd1) < 0x1p400)) rd1 = 0.0;
    // lanes whose coordinate exists and can ever move (a zero diagonal never moves)
    const uint64_t live0 = __ballot(has0 && qd0 != 0.0), live1 = __ballot(has1 && qd1 != 0.0);
    // the wave's largest of a non-negative per-lane double (fmax: order-free, NaN-ignoring)
    auto wave_max = [](double v) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v = __builtin_fmax(v, __shfl_xor(v, o, 64));
        return v;
    };
    // sklearn's step of coordinate j from its lane's values (oracle/lasso_oracle.c):
    // H[j] after the first axpy is lane j's own fma (r = Q[j][j] there), then
    // fsign(tmp) * fmax(|tmp| - alpha, 0) / (qii + beta) by Markstein's correction (above) with its first
    // product as m * (fsign(tmp) * r): the sign is exact (+-1, or 0 with m = 0), so that product
    // is the same double and the sign multiply leaves the chain.  Returns lane cl's weight,
    // broadcast.  The IEEE-division branch is decided on that broadcast (scalar exponent test, no
    // vector compare on the chain): a quotient whose exponent is inside [2^-398, 2^399) has its
    // first product inside (2^-400, 2^400), where the Markstein step is the IEEE quotient; any
    // other (zero -- a zero numerator, or r = 0 for a divisor without a normal reciprocal --
    // subnormal, huge, inf, NaN) takes the division.  Both give the correctly rounded quotient
    // wherever both apply, so the narrower test changes no bit.
    auto solve = [&](double qv, double hv, double wv, double qdv, double ddv, double rdv, int cl) {
        // (with a zero weight: fma(-+0, qii, h) differs from h at most in the sign of a zero h,
        // which changes tmp only between +0 and -0 -- the same weight either way)
        const double hh = __builtin_fma(-wv, qdv, hv);
        const double tmp = qv - hh;
        const double m = __builtin_fmax(__builtin_fabs(tmp) - alpha, 0.0);
        const double sg = fsign(tmp);
        const double num = sg * m;
        const double qt0 = m * (sg * rdv);
        const double et = __builtin_fma(-qt0, ddv, num);
        double wn = bcast(__builtin_fma(et, rdv, qt0), cl);
        const uint32_t ex = (uint32_t)(__builtin_bit_cast(uint64_t, wn) >> 52) & 0x7ffu;
        if (__builtin_expect(ex - (1023u - 398u) >= 797u, 0))
            wn = bcast(num == 0.0 ? num : num / ddv, cl);
        if constexpr (POS) {
            if ((__builtin_amdgcn_ballot_w64(tmp < 0) >> cl) & 1) wn = 0.0;
        }
        return wn;
    };
    // One half's part of a sweep: coordinates are visited in increasing order, so a sweep runs
    // all moves of features 0..63, then all of 64..; within a half the step runs on that half's
    // registers in every lane at once (lane c's result kept): its weight, H, q, diagonal and
    // reciprocal are already there.  Each scan over the half's lanes above the last move records
    // the sign of q - h (ZN: what a lane skipped there stores) and finds the next movable one
    // (with its nonzero diagonal: w != 0, or the soft threshold of q - h is nonzero --
    // fmax(|t| - alpha, 0) != 0 is |t| > alpha, NaN: false).  Coordinates that cannot move are
    // exactly sklearn's no-ops.
    auto half = [&](double& qh, double& hh, double& wh, double qdh, double ddh, double rdh,
                    uint64_t liveh, uint64_t& ZN, int base) {
        uint64_t ab = ~0ull;                 // the half's lanes above the last move
        auto scan = [&]() -> uint64_t {
            const double t = qh - hh;
            if constexpr (!POS) ZN ^= (ZN ^ __builtin_amdgcn_ballot_w64(t < 0.0)) & ab;
            return (__builtin_amdgcn_ballot_w64(wh != 0.0) |
                    __builtin_amdgcn_ballot_w64(POS ? t > alpha : __builtin_fabs(t) > alpha)) &
                   liveh & ab;
        };
        for (uint64_t mv = scan(); mv; mv = scan()) {
            const int cl = __builtin_amdgcn_readfirstlane(__builtin_ctzll(mv));
            // (the masks never name a coordinate with a zero diagonal: not movable)
            const double* row = Q + (base + cl) * kQS;   // (zero past column p: no lane masks)
            const double r0 = row[j0], r1 = row[j1];
            const double w_c = bcast(wh, cl);
            const double wn = solve(qh, hh, wh, qdh, ddh, rdh, cl);
            wh = lane == cl ? wn : wh;
            // the axpys run unconditionally: with a zero weight fma(+-0, r, h) = h for the finite
            // Gram (a zero h may change the sign of its zero, which reaches no weight: h enters
            // only through q - h and further fmas)
            h0 = __builtin_fma(wn, r0, __builtin_fma(-w_c, r0, h0));
            h1 = __builtin_fma(wn, r1, __builtin_fma(-w_c, r1, h1));
            ab = ~1ull << cl;
        }
    };
    for (n_iter = 0; n_iter < max_iter; ++n_iter) {
        // Each coordinate is visited once per sweep, so its d_w is |w at the sweep's end - w at
        // its start| and both maxima are taken once per sweep (fmax: the same values).  The
        // signed zero a skipped coordinate stores (sklearn's fsign(tmp) * 0 / (qii + beta)) is
        // the sign of q - h at its visit, i.e. after the last update before it (ZN), applied to
        // the lanes that were zero before and after their visit at the sweep's end.
        const double ws0 = w0, ws1 = w1;
        uint64_t ZN0 = 0, ZN1 = 0;
        half(q0, h0, w0, qd0, dd0, rd0, live0, ZN0, 0);
        half(q1, h1, w1, qd1, dd1, rd1, live1, ZN1, 64);
        if constexpr (!POS) {
            // zero before and after the visit (skipped): the sign of q - h there
            if (((live0 >> lane) & 1) && ws0 == 0.0 && w0 == 0.0) w0 = ((ZN0 >> lane) & 1) ? -0.0 : 0.0;
            if (((live1 >> lane) & 1) && ws1 == 0.0 && w1 == 0.0) w1 = ((ZN1 >> lane) & 1) ? -0.0 : 0.0;
        }
        const double d_w_max = wave_max(__builtin_fmax(__builtin_fabs(w0 - ws0), __builtin_fabs(w1 - ws1)));
        const double w_max = wave_max(__builtin_fmax(__builtin_fabs(w0), __builtin_fabs(w1)));
        if (w_max == 0.0 || d_w_max / w_max < d_w_tol || n_iter == max_iter - 1) {
            double q_dot_w = 0.0, wh = 0.0, w_norm2 = 0.0, asum = 0.0, dual = 0.0;
            for (int j = 0; j < p; ++j) {
                const double wj = pick(w0, w1, j), qj = pick(q0, q1, j), hj = pick(h0, h1, j);
                q_dot_w = q_dot_w + wj * qj;
                const double xta = qj - hj - beta * wj;
                const double a = POS ? xta : __builtin_fabs(xta);
                if (j == 0 || a > dual) dual = a;
                wh = wh + wj * hj;
                w_norm2 = w_norm2 + wj * wj;
                asum = asum + __builtin_fabs(wj);
            }
            const double r_norm2 = ynorm2 + wh - 2.0 * q_dot_w;
            double cst;
            if (dual > alpha) {
                cst = alpha / dual;
                const double a_norm2 = r_norm2 * (cst * cst);
                gap = 0.5 * (r_norm2 + a_norm2);
            } else {
                cst = 1.0;
                gap = r_norm2;
            }
            gap = gap + (alpha * asum - cst * ynorm2 + cst * q_dot_w +
                         0.5 * beta * (1 + cst * cst) * w_norm2);
            if (gap < tol_y) break;
        }
    }
    if (w_out) {
        if (has0) w_out[j0] = w0;
        if (has1) w_out[j1] = w1;
    }
    if (beta_out) {
        if (has0) beta_out[1 + j0] = w0;
        if (has1) beta_out[1 + j1] = w1;
        double xw = 0.0;                             // X_offset . w, feature order
        for (int j = 0; j < p; ++j)
            xw = xw + (shift[1 + j] + gram[1 + j] / n) * pick(w0, w1, j);
        if (lane == 0) beta_out[0] = (shift[1 + p] + gram[1 + p] / n) - xw;
    }
    if (lane == 0) {
        info[0] = gap;
        info[1] = tol_y;
        info[2] = (double)(n_iter < max_iter ? n_iter + 1 : max_iter);
    }
}

}  // namespace
}  // namespace afm

template <bool POS>
static int launch_cd_t(afm_ctx* ctx, int lds, const double* gram, int p, double alpha, double beta,
                       int max_iter, double tol, double* w, double* info, double alpha_row,
                       const double* shift, double* beta_out) {
    AFM_HIP(afm_lds_opt_in(ctx, (const void*)afm::lasso_cd_kernel<POS>,
                           (int)sizeof(double) * afm::kMaxLassoP * afm::kQS));
    hipLaunchKernelGGL(afm::lasso_cd_kernel<POS>, dim3(1), dim3(afm::kLassoThreads), lds,
                       ctx->stream, gram, p, alpha, beta, max_iter, tol, w, info, alpha_row, shift,
                       beta_out);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}
static int launch_cd(afm_ctx* ctx, bool positive, int lds, const double* gram, int p, double alpha,
                     double beta, int max_iter, double tol, double* w, double* info,
                     double alpha_row, const double* shift, double* beta_out) {
    return positive ? launch_cd_t<true>(ctx, lds, gram, p, alpha, beta, max_iter, tol, w, info,
                                        alpha_row, shift, beta_out)
                    : launch_cd_t<false>(ctx, lds, gram, p, alpha, beta, max_iter, tol, w, info,
                                         alpha_row, shift, beta_out);
}

extern "C" int afm_lasso_cd_f64(afm_ctx* ctx, const double* gram, int p, double alpha_n,
                                double beta, int max_iter, double tol, int positive, double* w,
                                double* info) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(p >= 1 && p <= afm::kMaxLassoP, "need 1 <= p <= 110");
    AFM_CHECK_ARG(gram && w && info, "null buffer");
    AFM_CHECK_ARG(max_iter >= 1, "max_iter must be >= 1");
    AFM_CHECK_ARG(alpha_n >= 0 && beta >= 0 && tol >= 0, "alpha, beta and tol must be >= 0");
    const int lds = (int)sizeof(double) * p * afm::kQS;
    return launch_cd(ctx, positive != 0, lds, gram, p, alpha_n, beta, max_iter, tol, w, info, -1.0,
                     nullptr, nullptr);
}

extern "C" int afm_lasso_fit_f64(afm_ctx* ctx, const double* gram, const double* shift, int p,
                                 double alpha, int max_iter, double tol, int positive,
                                 double* beta_out, double* info) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(p >= 1 && p <= afm::kMaxLassoP, "need 1 <= p <= 110");
    AFM_CHECK_ARG(gram && shift && beta_out && info, "null buffer");
    AFM_CHECK_ARG(max_iter >= 1 && alpha >= 0 && tol >= 0, "bad max_iter / alpha / tol");
    const int lds = (int)sizeof(double) * p * afm::kQS;
    return launch_cd(ctx, positive != 0, lds, gram, p, 0.0, 0.0, max_iter, tol, nullptr, info, alpha,
                     shift, beta_out);
}

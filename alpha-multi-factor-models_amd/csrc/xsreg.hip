// Cross-sectional regression: per-segment shifted Gram matrices on fp64
// MFMA, batched scaled-Cholesky OLS solves, the pooled (train+valid) OLS as an exact Chan
// combination of the per-segment moments, Fama-MacBeth statistics and predictions.
//
// A "segment" is the set of rows reduced into one Gram: one DATE of a calendar-grid panel
// (rows = the assets present that day, read straight from the factor planes), or one block of
// rows of a long design matrix (the LinearRegression drop-in, KKT:582-590).
//
// Gram kernel (one workgroup = 4 waves per segment):
//   Z = [1, x_1 .. x_p, y] over the segment's usable rows (mask bit set and every value finite),
//   shifted by the first usable row s (Z - s keeps the moments well conditioned; column 0 is
//   not shifted), G' = sum_rows (z - s)(z - s)^T.  Rows are staged 64 at a time through an LDS
//   tile [feature][row] (row stride 66 doubles -> conflict-free fragment reads) and reduced with
//   v_mfma_f64_16x16x4_f64 over the upper-triangle 16x16 tile pairs; waves split tile pairs
//   (wide designs) and/or rows (narrow designs), partial sums are combined in a fixed order, so
//   results are deterministic.
// Algorithmic work per segment: rows * (p+2)(p+3) flops over 8(p+1) B per row.
#include "afm_internal.h"

#pragma clang fp contract(off)

namespace afm {
namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;

constexpr int kMaxTiles = 7;          // p + 2 <= 112
constexpr int kMaxF = kMaxTiles * 16;
constexpr int kRS = 66;               // LDS tile row stride (doubles)
constexpr int kRows = 64;             // rows staged per tile
constexpr int kThreads = 256;

struct GramArgs {
    const double* base;      // planes / columns
    int64_t col_stride;      // elements between two columns
    int64_t seg_stride;      // elements between the first rows of two consecutive segments
    int64_t seg_rows;        // rows per segment
    int64_t row_limit;       // long mode: total rows (rows >= limit are masked); grid: -1
    const int32_t* cols;     // [p] column indices of the regressors
    int32_t ycol;            // column index of the regressand
    int p;
    const uint64_t* bits;    // grid mode: [ceil(T/64)][seg_stride] presence words; may be null
    int64_t seg0;            // first segment (date) index
    double* gram;            // [nseg][p2][p2]
    double* shift;           // [nseg][p2]
};

__device__ __forceinline__ int pair_I(int q, int nt) {
    int I = 0;
    while (q >= nt - I) { q -= nt - I; ++I; }
    return I;
}
__device__ __forceinline__ int pair_J(int q, int nt) {
    int I = 0;
    while (q >= nt - I) { q -= nt - I; ++I; }
    return I + q;
}

constexpr int kPer = ((kMaxF - 1) * kRows + kThreads - 1) / kThreads;   // staged values per thread

__global__ __launch_bounds__(kThreads) void gram_kernel(GramArgs g) {
    __shared__ double tile[kMaxF][kRS];
    __shared__ double sh[kMaxF];
    __shared__ int colsL[kMaxF];
    __shared__ int rowok[kRows];
    __shared__ int flags[2];               // [0] shift set, [1] tile has a usable row
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int p = g.p, p2 = p + 2;
    const int nt = (p2 + 15) / 16;
    const int npairs = nt * (nt + 1) / 2;
    // split 4 waves over tile pairs (WP) x row k-steps (WK)
    const int WP = npairs >= 8 ? 4 : (npairs >= 3 ? 2 : 1);
    const int WK = 4 / WP;
    const int wp = wave % WP, wk = wave / WP;
    const int64_t seg = g.seg0 + blockIdx.x;
    const int64_t rowbase = seg * g.seg_stride;
    const int nstage = (p + 1) * kRows;

    for (int i = tid; i < kMaxF * kRS; i += kThreads) (&tile[0][0])[i] = 0.0;
    if (tid < kMaxF) sh[tid] = 0.0;
    if (tid < p + 1) colsL[tid] = tid < p ? g.cols[tid] : g.ycol;
    if (tid == 0) flags[0] = 0;
    // this wave's tile pairs
    int pI[kMaxTiles], pJ[kMaxTiles];
#pragma unroll
    for (int q = 0; q < kMaxTiles; ++q) {
        const int pq = wp + q * WP;
        pI[q] = pq < npairs ? pair_I(pq, nt) : 0;
        pJ[q] = pq < npairs ? pair_J(pq, nt) : 0;
    }
    d4 acc[kMaxTiles];
#pragma unroll
    for (int q = 0; q < kMaxTiles; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
    __syncthreads();

    // register prefetch of one 64-row tile of features 1..p+1
    double pre[kPer];
    auto prefetch = [&](int64_t r0) {
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int i = tid + j * kThreads;
            double x = 0.0;
            if (i < nstage) {
                const int f = 1 + (i >> 6), a = i & (kRows - 1);
                const int64_t r = r0 + a;
                bool in = r < g.seg_rows;
                if (g.row_limit >= 0) in = in && (rowbase + r < g.row_limit);
                if (in) x = g.base[(int64_t)colsL[f - 1] * g.col_stride + rowbase + r];
            }
            pre[j] = x;
        }
    };
    prefetch(0);

    for (int64_t r0 = 0; r0 < g.seg_rows; r0 += kRows) {
        // ---- row mask of rows r0..r0+63, stage the prefetched values ----
        if (tid < kRows) {
            int64_t r = r0 + tid;
            bool ok = r < g.seg_rows;
            if (ok && g.row_limit >= 0) ok = rowbase + r < g.row_limit;
            if (ok && g.bits) {
                u64 w = g.bits[(seg >> 6) * g.seg_stride + r];
                ok = (w >> (seg & 63)) & 1ull;
            }
            rowok[tid] = ok ? 1 : 0;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int i = tid + j * kThreads;
            if (i < nstage) {
                const int f = 1 + (i >> 6), a = i & (kRows - 1);
                const double x = pre[j];
                if (rowok[a] && !__builtin_isfinite(x)) rowok[a] = 0;   // benign race: stores 0
                tile[f][a] = x;
            }
        }
        __syncthreads();
        if (r0 + kRows < g.seg_rows) prefetch(r0 + kRows);           // in flight during MFMA
        if (wave == 0) {
            u64 m = __ballot(rowok[lane] != 0);
            if (lane == 0) flags[1] = m != 0ull;
            if (m != 0ull && flags[0] == 0) {
                int a0 = __builtin_ctzll(m);
                for (int f = 1 + lane; f < p2; f += 64) sh[f] = tile[f][a0];
                if (lane == 0) flags[0] = 1;
            }
        }
        __syncthreads();
        if (!flags[1]) continue;                   // uniform: nothing usable in this tile
        for (int i = tid; i < p2 * kRows; i += kThreads) {
            int f = i >> 6, a = i & (kRows - 1);
            double v = 0.0;
            if (rowok[a]) v = (f == 0) ? 1.0 : tile[f][a] - sh[f];
            tile[f][a] = v;
        }
        __syncthreads();
        // ---- MFMA: acc[pair] += Z[:, I]^T Z[:, J] over this wave's k-steps ----
        const int fi = lane & 15, kk = lane >> 4;
        for (int ks = wk; ks < kRows / 4; ks += WK) {
            const int a = ks * 4 + kk;
#pragma unroll
            for (int q = 0; q < kMaxTiles; ++q) {
                if (wp + q * WP < npairs) {
                    const double va = tile[pI[q] * 16 + fi][a];
                    const double vb = tile[pJ[q] * 16 + fi][a];
                    acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(va, vb, acc[q], 0, 0, 0);
                }
            }
        }
        __syncthreads();
    }

    // ---- combine the WK row-groups in a fixed order, write G' (full symmetric) ----
    double* out = g.gram + (int64_t)blockIdx.x * p2 * p2;
    double* red = &tile[0][0];               // reuse: [WK][WP][kMaxTiles][64 lanes][4]
    auto slot = [&](int k_, int q_, int r_) {
        return (((k_ * WP + wp) * kMaxTiles + q_) * 64 + lane) * 4 + r_;
    };
    if (WK > 1) {
        for (int q = 0; q < kMaxTiles; ++q)
            for (int r = 0; r < 4; ++r) red[slot(wk, q, r)] = acc[q][r];
        __syncthreads();
    }
    if (wk == 0) {
        for (int q = 0; q < kMaxTiles; ++q) {
            const int pq = wp + q * WP;
            if (pq >= npairs) continue;
            const int I = pI[q], J = pJ[q];
            for (int r = 0; r < 4; ++r) {
                double v = acc[q][r];
                for (int k = 1; k < WK; ++k) v += red[slot(k, q, r)];
                const int row = I * 16 + (lane >> 4) + 4 * r;   // f64 MFMA C/D layout
                const int col = J * 16 + (lane & 15);
                if (row < p2 && col < p2) {
                    out[row * p2 + col] = v;
                    out[col * p2 + row] = v;
                }
            }
        }
    }
    if (tid < p2) g.shift[(int64_t)blockIdx.x * p2 + tid] = sh[tid];
}

// ---- per-segment OLS from the shifted Gram -------------------------------------------------
// C = G'[1:,1:] - G'[0,1:] G'[0,1:]^T / n (centered moments of [x, y]); scale to unit diagonal,
// Cholesky with a relative pivot threshold (a pivot below tol drops the regressor: beta = 0),
// beta = D b, intercept = ybar - xbar . beta.  One workgroup per segment, matrices in LDS.
struct SolveArgs {
    const double* gram;      // [nseg][p2][p2]
    const double* shift;     // [nseg][p2]
    int p;
    double tol;
    double* beta;            // [nseg][p+1]: intercept, beta_1..p
    double* nobs;            // [nseg]
    int32_t* rank;           // [nseg]
};

constexpr int kMaxP = kMaxF - 2;

__global__ __launch_bounds__(kThreads) void ols_solve_kernel(SolveArgs s) {
    __shared__ double M[kMaxP][kMaxP + 1];
    __shared__ double rhs[kMaxP];
    __shared__ double dsc[kMaxP];
    __shared__ double mean[kMaxP + 2];
    __shared__ int drop[kMaxP];
    __shared__ double piv;
    const int tid = threadIdx.x;
    const int p = s.p, p2 = p + 2;
    const double* G = s.gram + (int64_t)blockIdx.x * p2 * p2;
    const double* sf = s.shift + (int64_t)blockIdx.x * p2;
    const double n = G[0];
    double* beta = s.beta + (int64_t)blockIdx.x * (p + 1);
    if (tid == 0) s.nobs[blockIdx.x] = n;
    if (!(n > (double)p)) {                          // under-determined segment
        for (int j = tid; j <= p; j += kThreads) beta[j] = __builtin_nan("");
        if (tid == 0) s.rank[blockIdx.x] = 0;
        return;
    }
    for (int j = tid; j < p2; j += kThreads) mean[j] = (j == 0) ? 1.0 : G[j] / n;   // shifted
    __syncthreads();
    for (int i = tid; i < p * p; i += kThreads) {
        int r = i / p, c = i % p;
        M[r][c] = G[(r + 1) * p2 + (c + 1)] - G[r + 1] * G[c + 1] / n;
    }
    for (int r = tid; r < p; r += kThreads) rhs[r] = G[(r + 1) * p2 + (p + 1)] - G[r + 1] * G[p + 1] / n;
    __syncthreads();
    for (int r = tid; r < p; r += kThreads) {
        double d = M[r][r];
        dsc[r] = d > 0 ? 1.0 / __builtin_sqrt(d) : 0.0;
        drop[r] = !(d > 0);
    }
    __syncthreads();
    for (int i = tid; i < p * p; i += kThreads) {
        int r = i / p, c = i % p;
        M[r][c] = M[r][c] * dsc[r] * dsc[c];
    }
    for (int r = tid; r < p; r += kThreads) rhs[r] = rhs[r] * dsc[r];
    __syncthreads();
    // right-looking Cholesky (lower), thresholded
    for (int k = 0; k < p; ++k) {
        if (tid == 0) {
            double d = M[k][k];
            if (drop[k] || !(d > s.tol)) {
                drop[k] = 1;
                piv = 0.0;
            } else {
                piv = __builtin_sqrt(d);
            }
        }
        __syncthreads();
        const double pk = piv;
        if (pk == 0.0) {
            for (int i = tid; i < p; i += kThreads) { M[i][k] = 0.0; M[k][i] = 0.0; }
            __syncthreads();
            continue;
        }
        for (int i = k + tid; i < p; i += kThreads) M[i][k] = (i == k) ? pk : M[i][k] / pk;
        __syncthreads();
        const int m = p - k - 1;
        for (int e = tid; e < m * m; e += kThreads) {
            int i = k + 1 + e / m, j = k + 1 + e % m;
            if (j <= i) M[i][j] = M[i][j] - M[i][k] * M[j][k];
        }
        __syncthreads();
    }
    // forward / back substitution (sequential in k; every wave takes part in the barriers)
    for (int k = 0; k < p; ++k) {
        if (tid == 0) rhs[k] = drop[k] ? 0.0 : rhs[k] / M[k][k];
        __syncthreads();
        const double v = rhs[k];
        for (int i = k + 1 + tid; i < p; i += kThreads) rhs[i] = rhs[i] - M[i][k] * v;
        __syncthreads();
    }
    for (int k = p - 1; k >= 0; --k) {
        if (tid == 0) rhs[k] = drop[k] ? 0.0 : rhs[k] / M[k][k];
        __syncthreads();
        const double v = rhs[k];
        for (int i = tid; i < k; i += kThreads) rhs[i] = rhs[i] - M[k][i] * v;
        __syncthreads();
    }
    if (tid == 0) {
        double icpt = sf[p + 1] + mean[p + 1];           // ybar
        int rk = 0;
        for (int j = 0; j < p; ++j) {
            double b = rhs[j] * dsc[j];
            beta[1 + j] = b;
            icpt = icpt - (sf[1 + j] + mean[1 + j]) * b;
            rk += drop[j] ? 0 : 1;
        }
        beta[0] = icpt;
        s.rank[blockIdx.x] = rk;
    }
}

// ---- exact (Chan) combination of per-segment shifted moments ----------------------------------
// Block b combines segments [b*per, min((b+1)*per, nseg)) in order and emits the union's moments
// in the same "shifted" representation (G'[0][0] = n, G'[0][j] = 0, G'[i][j] = centered sums,
// shift = mean), so a second pass (or ols_solve_kernel) consumes it unchanged.  Two passes with
// per = 64 give the same tree for any split of the segments into 64-aligned shards (multi-GPU).
constexpr int kPoolBlock = 64;

__global__ __launch_bounds__(kThreads) void pool_kernel(const double* gram, const double* shift,
                                                        int p2, int64_t nseg, int64_t per,
                                                        double* out_gram, double* out_shift) {
    extern __shared__ __attribute__((aligned(16))) double C[];   // [p2][p2]
    __shared__ double mu[kMaxF];
    __shared__ double dl[kMaxF];
    __shared__ double ntot_s, fac_s;
    const int tid = threadIdx.x;
    const int q2 = p2 * p2;
    const int64_t s0 = (int64_t)blockIdx.x * per;
    const int64_t s1 = s0 + per < nseg ? s0 + per : nseg;
    for (int e = tid; e < q2; e += kThreads) C[e] = 0.0;
    if (tid < p2) mu[tid] = 0.0;
    if (tid == 0) ntot_s = 0.0;
    __syncthreads();
    for (int64_t sg = s0; sg < s1; ++sg) {
        const double* G = gram + sg * q2;
        const double* S = shift + sg * p2;
        const double nb = G[0];
        if (!(nb > 0)) continue;                       // uniform
        if (tid < p2 && tid > 0) dl[tid] = (S[tid] + G[tid] / nb) - mu[tid];
        if (tid == 0) {
            const double na = ntot_s;
            fac_s = na * nb / (na + nb);
            ntot_s = na + nb;
        }
        __syncthreads();
        const double fac = fac_s;
        for (int e = tid; e < q2; e += kThreads) {
            const int r = e / p2, c = e - r * p2;
            if (r > 0 && c > 0) {
                const double cb = G[e] - G[r] * G[c] / nb;            // segment centered
                C[e] = C[e] + cb + dl[r] * dl[c] * fac;
            }
        }
        __syncthreads();
        if (tid < p2 && tid > 0) mu[tid] = mu[tid] + dl[tid] * (nb / ntot_s);
        __syncthreads();
    }
    double* og = out_gram + (int64_t)blockIdx.x * q2;
    for (int e = tid; e < q2; e += kThreads) {
        const int r = e / p2, c = e - r * p2;
        og[e] = (r == 0 && c == 0) ? ntot_s : ((r == 0 || c == 0) ? 0.0 : C[e]);
    }
    if (tid < p2) out_shift[(int64_t)blockIdx.x * p2 + tid] = (tid == 0) ? 0.0 : mu[tid];
}

// ---- predictions: pred[t][a] = beta0 + sum_j beta_j x_j (grid rows with a set mask bit) ------
__global__ __launch_bounds__(256) void predict_kernel(const double* base, int64_t col_stride,
                                                      int64_t lda, int64_t t0, int64_t nt,
                                                      const int32_t* cols, int p,
                                                      const double* beta, int64_t beta_stride,
                                                      const uint64_t* bits, int ycheck,
                                                      double* pred) {
    const int64_t a = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    const int64_t t = t0 + (int64_t)blockIdx.y * 4 + (threadIdx.x >> 6);
    if (t >= t0 + nt) return;
    const double* b = beta + (t - t0) * beta_stride;
    u64 w = bits[(t >> 6) * lda + a];
    double v = __builtin_nan("");
    bool use = (w >> (t & 63)) & 1ull;
    if (use && ycheck >= 0) use = __builtin_isfinite(base[(int64_t)ycheck * col_stride + t * lda + a]);
    if (use) {
        double s = b[0];
        for (int j = 0; j < p; ++j) s = s + b[1 + j] * base[(int64_t)cols[j] * col_stride + t * lda + a];
        v = s;
    }
    pred[t * lda + a] = v;
}

// ---- least-squares refinement: r = (y - ybar) - sum_j b_j (x_j - xbar_j) over a long design ----
__global__ __launch_bounds__(256) void residual_kernel(const double* Z, int64_t n, int p, int ycol,
                                                       const double* mean, const double* beta,
                                                       double* r) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double s = Z[(int64_t)ycol * n + i] - mean[p + 1];
    for (int j = 0; j < p; ++j) s = s - beta[1 + j] * (Z[(int64_t)j * n + i] - mean[1 + j]);
    r[i] = s;
}

__global__ void vec_add_kernel(int64_t n, const double* x, double* y) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) y[i] = y[i] + x[i];
}

__global__ void intercept_kernel(int p, const double* mean, double* beta) {
    if (threadIdx.x != 0) return;
    double icpt = mean[p + 1];
    for (int j = 0; j < p; ++j) icpt = icpt - mean[1 + j] * beta[1 + j];
    beta[0] = icpt;
}

// ---- Fama-MacBeth: mean_t beta_t and t = mean / (std / sqrt(T)) over segments with rank > 0 --
// One workgroup per coefficient: two passes (sum, then squared deviations from the mean), each a
// strided per-thread sum followed by a fixed-order tree over the 256 threads (deterministic).
__device__ double block_sum256(double v, double* red) {
    const int tid = threadIdx.x;
    red[tid] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) red[tid] = red[tid] + red[tid + o];
        __syncthreads();
    }
    const double r = red[0];
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(256) void fama_macbeth_kernel(const double* beta, const int32_t* rank,
                                                           int64_t nseg, int k, double* mean_out,
                                                           double* t_out) {
    __shared__ double red[256];
    const int j = blockIdx.x, tid = threadIdx.x;
    double n = 0, s = 0;
    for (int64_t q = tid; q < nseg; q += 256)
        if (rank[q] > 0) { n += 1; s += beta[q * k + j]; }
    n = block_sum256(n, red);
    s = block_sum256(s, red);
    const double m = s / n;
    double ss = 0;
    for (int64_t q = tid; q < nseg; q += 256)
        if (rank[q] > 0) { const double d = beta[q * k + j] - m; ss += d * d; }
    ss = block_sum256(ss, red);
    if (tid == 0) {
        const double sd = n > 1 ? __builtin_sqrt(ss / (n - 1)) : __builtin_nan("");
        mean_out[j] = n > 0 ? m : __builtin_nan("");
        t_out[j] = m / (sd / __builtin_sqrt(n));
    }
}

}  // namespace
}  // namespace afm

using namespace afm;

extern "C" int afm_xs_gram_f64(afm_ctx* ctx, const double* base, int64_t col_stride,
                               int64_t seg_stride, int64_t seg_rows, int64_t row_limit,
                               const int32_t* cols, int p, int ycol, const uint64_t* bits,
                               int64_t seg0, int64_t nseg, double* gram, double* shift) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(p >= 1 && p + 2 <= kMaxF, "need 1 <= p <= 110");
    AFM_CHECK_ARG(base && cols && gram && shift, "null buffer");
    AFM_CHECK_ARG(nseg >= 0 && seg0 >= 0 && seg_rows > 0, "bad segment range");
    AFM_CHECK_ARG(!bits || seg_stride % 64 == 0, "grid mode needs seg_stride (lda) % 64 == 0");
    if (nseg == 0) return AFM_OK;
    GramArgs g{base, col_stride, seg_stride, seg_rows, row_limit, cols, ycol, p, bits, seg0, gram,
               shift};
    hipLaunchKernelGGL(gram_kernel, dim3((unsigned)nseg), dim3(kThreads), 0, ctx->stream, g);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_ols_solve_f64(afm_ctx* ctx, const double* gram, const double* shift, int p,
                                 int64_t nseg, double tol, double* beta, double* nobs,
                                 int32_t* rank) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(p >= 1 && p <= kMaxP, "need 1 <= p <= 110");
    AFM_CHECK_ARG(gram && shift && beta && nobs && rank, "null buffer");
    if (nseg <= 0) return AFM_OK;
    SolveArgs s{gram, shift, p, tol, beta, nobs, rank};
    hipLaunchKernelGGL(ols_solve_kernel, dim3((unsigned)nseg), dim3(kThreads), 0, ctx->stream, s);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_pool_moments_f64(afm_ctx* ctx, const double* gram, const double* shift, int p,
                                    int64_t nseg, double* out_gram, double* out_shift) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(p >= 1 && p + 2 <= kMaxF, "need 1 <= p <= 110");
    AFM_CHECK_ARG(gram && shift && out_gram && out_shift && nseg >= 0, "bad arguments");
    const int p2 = p + 2;
    const size_t lds = sizeof(double) * p2 * p2;
    AFM_HIP(hipFuncSetAttribute((const void*)pool_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int64_t nb = (nseg + kPoolBlock - 1) / kPoolBlock;
    if (nb <= 1) {
        hipLaunchKernelGGL(pool_kernel, dim3(1), dim3(kThreads), lds, ctx->stream, gram, shift,
                           p2, nseg, (int64_t)kPoolBlock, out_gram, out_shift);
        AFM_HIP(hipGetLastError());
        return AFM_OK;
    }
    double* work = nullptr;
    AFM_HIP(hipMallocAsync((void**)&work, sizeof(double) * nb * (p2 * p2 + p2), ctx->stream));
    double* wg = work;
    double* ws = work + nb * p2 * p2;
    hipLaunchKernelGGL(pool_kernel, dim3((unsigned)nb), dim3(kThreads), lds, ctx->stream, gram,
                       shift, p2, nseg, (int64_t)kPoolBlock, wg, ws);
    AFM_HIP(hipGetLastError());
    hipLaunchKernelGGL(pool_kernel, dim3(1), dim3(kThreads), lds, ctx->stream, wg, ws, p2, nb, nb,
                       out_gram, out_shift);
    AFM_HIP(hipGetLastError());
    AFM_HIP(hipFreeAsync(work, ctx->stream));
    return AFM_OK;
}

extern "C" int afm_predict_f64(afm_ctx* ctx, const double* base, int64_t col_stride, int64_t lda,
                               int64_t t0, int64_t nt, const int32_t* cols, int p,
                               const double* beta, int64_t beta_stride, const uint64_t* bits,
                               int ycheck, double* pred) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(base && cols && beta && bits && pred, "null buffer");
    AFM_CHECK_ARG(lda % 64 == 0 && nt >= 0 && t0 >= 0, "bad shape");
    if (nt == 0) return AFM_OK;
    dim3 grid((unsigned)(lda / 64), (unsigned)((nt + 3) / 4));
    hipLaunchKernelGGL(predict_kernel, grid, dim3(256), 0, ctx->stream, base, col_stride, lda, t0,
                       nt, cols, p, beta, beta_stride, bits, ycheck, pred);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_fama_macbeth_f64(afm_ctx* ctx, const double* beta, const int32_t* rank,
                                    int64_t nseg, int k, double* mean_out, double* t_out) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(beta && rank && mean_out && t_out && k > 0, "bad args");
    hipLaunchKernelGGL(fama_macbeth_kernel, dim3(k), dim3(256), 0, ctx->stream, beta,
                       rank, nseg, k, mean_out, t_out);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_ols_residual_f64(afm_ctx* ctx, const double* Z, int64_t n, int p, int ycol,
                                    const double* mean, const double* beta, double* r) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(Z && mean && beta && r && n >= 0 && p >= 1, "bad arguments");
    if (n == 0) return AFM_OK;
    hipLaunchKernelGGL(residual_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       ctx->stream, Z, n, p, ycol, mean, beta, r);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_vec_add_f64(afm_ctx* ctx, int64_t n, const double* x, double* y) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(x && y && n >= 0, "bad arguments");
    if (n == 0) return AFM_OK;
    hipLaunchKernelGGL(vec_add_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       ctx->stream, n, x, y);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_ols_intercept_f64(afm_ctx* ctx, int p, const double* mean, double* beta) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(mean && beta && p >= 1, "bad arguments");
    hipLaunchKernelGGL(intercept_kernel, dim3(1), dim3(64), 0, ctx->stream, p, mean, beta);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

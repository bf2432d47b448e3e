// Rebalance + weights + PnL: PortfolioManager.calculate_portfolio
// ("KKT Yuliang Jiang.py":842-892) with the exact box-constrained min-variance solve.
//
// rebalance_kernel -- one workgroup (256 threads) per rebalance date:
//   1. candidates = assets with a prediction (non-NaN) that are tradable that day (KKT:847-848);
//      k = n//2 on thin dates, else top_n (KKT:849-852);
//   2. long = k largest predictions (descending), short = k smallest (ascending); ties broken by
//      ascending asset index (the reference breaks them in Python-set order, KKT:855-856).
//      Exact radix select on order-preserving 64-bit keys, then a rank-by-count sort of the k;
//   3. per book, the pairwise-complete covariance of the members' history returns over the
//      history window (KKT:858-859, 821-822: pandas nancorr(cov=True) Welford, rows in date
//      order), one thread per member pair, history staged through LDS 64 dates at a time;
//   4. min w'Sw  s.t. sum w = 1, lo <= w <= hi (KKT:811-833) solved EXACTLY by a primal
//      active-set method: each step solves the KKT system [S_FF 1; 1' 0][w_F; lam] by an LDS
//      Cholesky of S_FF and the Schur complement of the equality (SLSQP is not a parity target,
//      SURVEY.md §0 F6);
//   5. per book: sum(tmr * w) as numpy's pairwise sum (Series.sum, KKT:875-877) and
//      sum(w * close) as Python's sequential builtin sum (KKT:881-882); the members' positions
//      in the id-union of this and the neighbouring rebalance dates' prediction sets (the
//      alignment of KKT:839) for the turnover scan.
// pnl_scan_kernel -- one thread: the value/turnover recursion over the rebalance dates
//   (KKT:864-892), turnover = numpy pairwise sum over the aligned union vector (zeros and NaN
//   -> 0 included, evaluated sparsely at the members' union positions).
#include "afm_internal.h"

#pragma clang fp contract(off)

namespace afm {
namespace {

typedef unsigned long long u64;
constexpr int kT = 256;        // threads per workgroup
constexpr int kMaxK = 64;      // max book size handled in LDS
constexpr int kMaxWords = 512; // lda <= 32768 assets

struct RebArgs {
    int64_t T, lda, A;
    const int32_t* dates;     // [nd] grid date index of each rebalance date (ascending)
    int64_t nd;
    const double* pred;       // [T][lda] NaN = no prediction
    const uint64_t* trad;     // [nch][lda] tradable bits (present in all_df AND 'Y')
    const double* hist;       // [T][lda] history returns (df_train_y target)
    const uint64_t* hbits;    // [nch][lda] history presence
    int64_t h_t0, h_t1;       // fixed history range [h_t0, h_t1) when window <= 0
    int64_t window;           // > 0: rolling window of `window` dates before the rebalance date
    const double* close;      // [T][lda]
    const double* tmr;        // [T][lda]
    int top_n;
    double lo, hi;
    // outputs (per rebalance date i)
    int32_t* k_out;           // [nd]
    int32_t* books;           // [nd][2][kMaxK] asset indices (long book, short book)
    double* weights;          // [nd][2][kMaxK]
    double* sums;             // [nd][4]: long_ret, short_ret, den_long, den_short
    int32_t* upos;            // [nd][2][2][kMaxK]: union position vs prev / vs next (-1 absent)
    int64_t* usize;           // [nd][2]: |P_prev U P_i|, |P_i U P_next|
    int32_t* status;          // [nd]: 0 ok, 1 QP iteration cap, 2 k > kMaxK
};

__device__ __forceinline__ u64 okey(double v) {   // order-preserving key, -0.0 == +0.0
    if (v == 0.0) v = 0.0;
    u64 u = (u64)__double_as_longlong(v);
    return (u >> 63) ? ~u : (u | (1ull << 63));
}

__device__ __forceinline__ bool bit_at(const uint64_t* bits, int64_t lda, int64_t t, int64_t a) {
    return (bits[(t >> 6) * lda + a] >> (t & 63)) & 1ull;
}

// block-wide exclusive scan of one int per thread (256 threads); returns the total
__device__ int block_scan(int v, int* sbuf, int* excl) {
    const int tid = threadIdx.x;
    sbuf[tid] = v;
    __syncthreads();
    for (int off = 1; off < kT; off <<= 1) {
        int x = tid >= off ? sbuf[tid - off] : 0;
        __syncthreads();
        sbuf[tid] += x;
        __syncthreads();
    }
    *excl = sbuf[tid] - v;
    int total = sbuf[kT - 1];
    __syncthreads();
    return total;
}

struct Shared {
    u64 pw[3][kMaxWords];                // prediction presence rows: prev, cur, next
    int hist[256];
    int scan[kT];
    int misc[8];
    u64 keysel[2 * kMaxK];
    int idxsel[2 * kMaxK];
    int book[2][kMaxK];
    double S[kMaxK][kMaxK + 1];          // covariance of the current book
    double L[kMaxK][kMaxK + 1];          // Cholesky work
    double hv[kMaxK][65];                // staged history chunk [member][date]
    double w[kMaxK], x[kMaxK], y1[kMaxK], y2[kMaxK], c[kMaxK], g[kMaxK];
    int state[kMaxK], F[kMaxK];
    double red[8];
};

// k largest keys among candidates (key valid when cand), ties -> smaller index first.
// Writes the selected indices, sorted (key desc, index asc), to out[0..k).
__device__ void select_top(const RebArgs& r, Shared& sh, int64_t t, int k, bool largest, int* out) {
    const int tid = threadIdx.x;
    const int64_t A = r.A;
    u64 prefix = 0, pmask = 0;
    int need = k;
    for (int shift = 56; shift >= 0; shift -= 8) {
        sh.hist[tid] = 0;
        __syncthreads();
        for (int64_t a = tid; a < A; a += kT) {
            double v = r.pred[t * r.lda + a];
            if (v == v && bit_at(r.trad, r.lda, t, a)) {
                u64 kk = okey(v);
                if (!largest) kk = ~kk;
                if ((kk & pmask) == prefix) atomicAdd(&sh.hist[(kk >> shift) & 255], 1);
            }
        }
        __syncthreads();
        if (tid == 0) {
            int acc = 0, d = 255;
            for (; d > 0; --d) {
                if (acc + sh.hist[d] >= need) break;
                acc += sh.hist[d];
            }
            sh.misc[0] = d;
            sh.misc[1] = need - acc;
        }
        __syncthreads();
        prefix |= (u64)sh.misc[0] << shift;
        pmask |= 255ull << shift;
        need = sh.misc[1];
        __syncthreads();
    }
    // prefix = threshold key tau; take all keys > tau and the first `need` equal ones by index
    int cnt_sel = 0, eq_seen = 0;           // uniform across the block
    for (int64_t base = 0; base < A; base += kT) {
        const int64_t a = base + tid;
        int eq = 0, gt = 0;
        u64 kk = 0;
        if (a < A) {
            double v = r.pred[t * r.lda + a];
            if (v == v && bit_at(r.trad, r.lda, t, a)) {
                kk = okey(v);
                if (!largest) kk = ~kk;
                gt = kk > prefix;
                eq = kk == prefix;
            }
        }
        int ex_eq, ex_t;
        const int tot_eq = block_scan(eq, sh.scan, &ex_eq);
        const bool take = gt || (eq && eq_seen + ex_eq < need);
        const int tot_t = block_scan(take ? 1 : 0, sh.scan, &ex_t);
        if (take) {
            sh.keysel[cnt_sel + ex_t] = kk;
            sh.idxsel[cnt_sel + ex_t] = (int)a;
        }
        cnt_sel += tot_t;
        eq_seen += tot_eq;
    }
    __syncthreads();
    // sort the k selected by (key desc, index asc): rank by counting
    if (tid < k) {
        u64 mk = sh.keysel[tid];
        int mi = sh.idxsel[tid];
        int rank = 0;
        for (int j = 0; j < k; ++j) {
            u64 ok = sh.keysel[j];
            int oi = sh.idxsel[j];
            rank += (ok > mk) || (ok == mk && oi < mi);
        }
        out[rank] = mi;
    }
    __syncthreads();
}

// numpy pairwise sum of a dense vector (n small)
__device__ double pairwise_dense(const double* a, int n) {
    if (n < 8) {
        double res = 0.;
        for (int i = 0; i < n; ++i) res += a[i];
        return res;
    } else if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    return pairwise_dense(a, n2) + pairwise_dense(a + n2, n - n2);
}

// min w'Sw  s.t. sum w = 1, lo <= w <= hi for the n x n matrix in sh.S -> sh.w.  Primal active
// set; each iteration solves [S_FF 1; 1' 0][w_F; lam] = [-S_FB w_B; b] by an LDS Cholesky of
// S_FF and the Schur complement of the equality.  Returns true if the iteration cap was hit.
// Called by every thread of the block.
__device__ bool qp_solve(Shared& sh, const int n, const double lo, const double hi) {
    const int tid = threadIdx.x;
    bool capped = false;
    if (n > 0 && n * hi <= 1.0) {
        if (tid < n) sh.w[tid] = hi;
    } else if (n > 0 && n * lo >= 1.0) {
        if (tid < n) sh.w[tid] = lo;
    } else if (n > 0) {
        if (tid < n) { sh.w[tid] = 1.0 / n; sh.state[tid] = 0; }
        __syncthreads();
        const int max_it = 4 * n + 8;
        for (int it = 0; it < max_it; ++it) {
            if (tid == 0) {
                int nf = 0;
                double bsum = 0.0;
                for (int q = 0; q < n; ++q) {
                    if (sh.state[q] == 0) sh.F[nf++] = q;
                    else bsum = bsum + sh.w[q];
                }
                sh.misc[5] = nf;
                sh.red[0] = 1.0 - bsum;
            }
            __syncthreads();
            const int nf = sh.misc[5];
            if (nf == 0) break;
            if (it == max_it - 1) capped = true;
            for (int e = tid; e < nf * nf; e += kT) {
                int a = e / nf, b = e % nf;
                sh.L[a][b] = sh.S[sh.F[a]][sh.F[b]];
            }
            if (tid < nf) {
                double cc = 0.0;
                for (int q = 0; q < n; ++q)
                    if (sh.state[q] != 0) cc = cc + sh.S[sh.F[tid]][q] * sh.w[q];
                sh.c[tid] = cc;
                sh.y1[tid] = 1.0;
                sh.y2[tid] = cc;
            }
            __syncthreads();
            for (int kk = 0; kk < nf; ++kk) {
                if (tid == 0) sh.L[kk][kk] = __builtin_sqrt(sh.L[kk][kk]);
                __syncthreads();
                for (int a = kk + 1 + tid; a < nf; a += kT) sh.L[a][kk] = sh.L[a][kk] / sh.L[kk][kk];
                __syncthreads();
                const int m = nf - kk - 1;
                for (int e = tid; e < m * m; e += kT) {
                    int a = kk + 1 + e / m, b = kk + 1 + e % m;
                    if (b <= a) sh.L[a][b] = sh.L[a][b] - sh.L[a][kk] * sh.L[b][kk];
                }
                __syncthreads();
            }
            if (tid < 2) {
                double* y = tid == 0 ? sh.y1 : sh.y2;
                for (int a = 0; a < nf; ++a) {
                    double s = y[a];
                    for (int b = 0; b < a; ++b) s = s - sh.L[a][b] * y[b];
                    y[a] = s / sh.L[a][a];
                }
                for (int a = nf - 1; a >= 0; --a) {
                    double s = y[a];
                    for (int b = a + 1; b < nf; ++b) s = s - sh.L[b][a] * y[b];
                    y[a] = s / sh.L[a][a];
                }
            }
            __syncthreads();
            if (tid == 0) {
                double s1 = 0.0, s2 = 0.0;
                for (int a = 0; a < nf; ++a) { s1 = s1 + sh.y1[a]; s2 = s2 + sh.y2[a]; }
                const double lam = -(sh.red[0] + s2) / s1;
                int feas = 1;
                for (int a = 0; a < nf; ++a) {
                    double xv = -sh.y2[a] - lam * sh.y1[a];
                    sh.x[a] = xv;
                    if (!(xv >= lo) || !(xv <= hi)) feas = 0;
                }
                int done = 0;
                if (feas) {
                    for (int a = 0; a < nf; ++a) sh.w[sh.F[a]] = sh.x[a];
                    int jmin = -1;
                    double vmin = 0.0;
                    for (int q = 0; q < n; ++q) {
                        if (sh.state[q] == 0) continue;
                        double gq = 0.0;
                        for (int b = 0; b < n; ++b) gq = gq + sh.S[q][b] * sh.w[b];
                        gq = gq + lam;
                        const double v = sh.state[q] < 0 ? gq : -gq;
                        if (v < vmin) { vmin = v; jmin = q; }
                    }
                    if (jmin < 0) done = 1;
                    else sh.state[jmin] = 0;
                } else {
                    double alpha = 1.0;
                    int jb = -1, bound = 0;
                    for (int a = 0; a < nf; ++a) {
                        const int q = sh.F[a];
                        const double pq = sh.x[a] - sh.w[q];
                        if (sh.x[a] < lo && pq < 0) {
                            const double al = (lo - sh.w[q]) / pq;
                            if (al < alpha) { alpha = al; jb = q; bound = -1; }
                        } else if (sh.x[a] > hi && pq > 0) {
                            const double al = (hi - sh.w[q]) / pq;
                            if (al < alpha) { alpha = al; jb = q; bound = 1; }
                        }
                    }
                    for (int a = 0; a < nf; ++a) {
                        const int q = sh.F[a];
                        sh.w[q] = sh.w[q] + alpha * (sh.x[a] - sh.w[q]);
                    }
                    if (jb >= 0) {
                        sh.w[jb] = bound < 0 ? lo : hi;
                        sh.state[jb] = bound;
                    }
                }
                sh.misc[7] = done;
            }
            __syncthreads();
            if (sh.misc[7]) break;
        }
    }
    __syncthreads();
    return capped;
}

// Welford pairwise-complete covariance (pandas nancorr, cov=True) of a dense [rows][ld] matrix
// (k columns, NaN = missing) into sh.S; rows staged 64 at a time.
__device__ void dense_cov(Shared& sh, const double* R, int64_t rows, int64_t ld, int k) {
    const int tid = threadIdx.x;
    const int npairs = k * (k + 1) / 2;
    for (int pb = 0; pb < npairs; pb += kT) {
        const int pq = pb + tid;
        int pi = 0, pj = 0;
        if (pq < npairs) {
            int q = pq;
            while (q > pi) { q -= pi + 1; ++pi; }
            pj = q;
        }
        double nobs = 0, mx = 0, my = 0, cxy = 0;
        for (int64_t h0 = 0; h0 < rows; h0 += 64) {
            __syncthreads();
            for (int e = tid; e < k * 64; e += kT) {
                const int m = e / 64, d = e % 64;
                sh.hv[m][d] = (h0 + d < rows) ? R[(h0 + d) * ld + m] : __builtin_nan("");
            }
            __syncthreads();
            if (pq < npairs) {
                const int nd = (int)((rows - h0) < 64 ? (rows - h0) : 64);
                for (int d = 0; d < nd; ++d) {
                    const double vx = sh.hv[pi][d], vy = sh.hv[pj][d];
                    if (__builtin_isfinite(vx) && __builtin_isfinite(vy)) {
                        nobs += 1;
                        const double dx = vx - mx, dy = vy - my;
                        mx += 1. / nobs * dx;
                        my += 1. / nobs * dy;
                        cxy += (vx - mx) * dy;
                    }
                }
            }
        }
        if (pq < npairs) {
            double cv = __builtin_nan("");
            if (nobs >= 1 && (nobs - 1.0) != 0) cv = cxy / (nobs - 1.0);
            sh.S[pi][pj] = cv;
            sh.S[pj][pi] = cv;
        }
    }
    __syncthreads();
}

__global__ __launch_bounds__(kT) void weights_kernel(const double* R, int64_t rows, int64_t ld,
                                                     int k, double lo, double hi, double* w,
                                                     double* cov, int32_t* status) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    Shared& sh = *reinterpret_cast<Shared*>(smem_raw);
    dense_cov(sh, R, rows, ld, k);
    const bool capped = qp_solve(sh, k, lo, hi);
    const int tid = threadIdx.x;
    if (tid < k) w[tid] = sh.w[tid];
    for (int e = tid; e < k * k; e += kT) cov[e] = sh.S[e / k][e % k];
    if (tid == 0) status[0] = capped ? 1 : 0;
}

__global__ __launch_bounds__(kT) void rebalance_kernel(RebArgs r) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    Shared& sh = *reinterpret_cast<Shared*>(smem_raw);
    const int tid = threadIdx.x;
    const int64_t i = blockIdx.x;
    const int64_t t = r.dates[i];
    const int64_t tp = i > 0 ? r.dates[i - 1] : -1;
    const int64_t tn = i + 1 < r.nd ? r.dates[i + 1] : -1;
    const int nw = (int)((r.A + 63) / 64);

    // ---- prediction presence rows (prev, cur, next) and candidate count --------------------
    for (int wi = tid; wi < nw; wi += kT) {
        u64 m[3] = {0, 0, 0};
        const int64_t ts[3] = {tp, t, tn};
        for (int q = 0; q < 3; ++q) {
            if (ts[q] < 0) continue;
            for (int b = 0; b < 64; ++b) {
                int64_t a = (int64_t)wi * 64 + b;
                if (a < r.A) {
                    double v = r.pred[ts[q] * r.lda + a];
                    if (v == v) m[q] |= 1ull << b;
                }
            }
        }
        for (int q = 0; q < 3; ++q) sh.pw[q][wi] = m[q];
    }
    int nc = 0;
    for (int64_t a = tid; a < r.A; a += kT) {
        double v = r.pred[t * r.lda + a];
        nc += (v == v && bit_at(r.trad, r.lda, t, a)) ? 1 : 0;
    }
    int ex;
    const int ncand = block_scan(nc, sh.scan, &ex);
    int k = ncand < 2 * r.top_n ? ncand / 2 : r.top_n;
    if (k > kMaxK) {
        if (tid == 0) { r.status[i] = 2; r.k_out[i] = k; }
        return;
    }
    if (tid == 0) { r.k_out[i] = k; r.status[i] = 0; }

    if (k > 0) {
        select_top(r, sh, t, k, true, sh.book[0]);
        select_top(r, sh, t, k, false, sh.book[1]);
    }
    __syncthreads();

    if (tid == 0) sh.misc[4] = 0;
    const int64_t hlo = r.window > 0 ? (t - r.window > 0 ? t - r.window : 0) : r.h_t0;
    const int64_t hhi = r.window > 0 ? t : r.h_t1;
    for (int side = 0; side < 2; ++side) {
        const int* bk = sh.book[side];
        // ---- pairwise-complete covariance (pandas nancorr, cov=True) ----------------------
        const int npairs = k * (k + 1) / 2;
        for (int pb = 0; pb < npairs; pb += kT) {
            const int pq = pb + tid;
            int pi = 0, pj = 0;
            if (pq < npairs) {   // pq -> (xi >= yi) in row-major lower-triangle order
                int q = pq;
                pi = 0;
                while (q > pi) { q -= pi + 1; ++pi; }
                pj = q;
            }
            double nobs = 0, mx = 0, my = 0, cxy = 0;
            for (int64_t h0 = hlo; h0 < hhi; h0 += 64) {
                __syncthreads();
                for (int e = tid; e < k * 64; e += kT) {
                    int m = e / 64, d = e % 64;
                    int64_t th = h0 + d;
                    double v = __builtin_nan("");
                    if (th < hhi && bit_at(r.hbits, r.lda, th, bk[m])) v = r.hist[th * r.lda + bk[m]];
                    sh.hv[m][d] = v;
                }
                __syncthreads();
                if (pq < npairs) {
                    const int nd = (int)((hhi - h0) < 64 ? (hhi - h0) : 64);
                    for (int d = 0; d < nd; ++d) {
                        double vx = sh.hv[pi][d], vy = sh.hv[pj][d];
                        if (__builtin_isfinite(vx) && __builtin_isfinite(vy)) {
                            nobs += 1;
                            double dx = vx - mx, dy = vy - my;
                            mx += 1. / nobs * dx;
                            my += 1. / nobs * dy;
                            cxy += (vx - mx) * dy;
                        }
                    }
                }
            }
            if (pq < npairs) {
                double cv = __builtin_nan("");
                if (nobs >= 1 && (nobs - 1.0) != 0) cv = cxy / (nobs - 1.0);
                sh.S[pi][pj] = cv;
                sh.S[pj][pi] = cv;
            }
        }
        __syncthreads();

        // ---- exact box-constrained QP (primal active set) --------------------------------
        if (qp_solve(sh, k, r.lo, r.hi) && tid == 0) sh.misc[4] = 1;
        __syncthreads();
        // ---- outputs for this book -------------------------------------------------------
        double* wout = r.weights + (i * 2 + side) * kMaxK;
        int32_t* bout = r.books + (i * 2 + side) * kMaxK;
        if (tid < k) {
            wout[tid] = sh.w[tid];
            bout[tid] = bk[tid];
            sh.x[tid] = r.tmr[t * r.lda + bk[tid]] * sh.w[tid];   // tmr * w (book order)
            sh.x[tid] = sh.x[tid] == sh.x[tid] ? sh.x[tid] : 0.0;  // nansum
            sh.c[tid] = sh.w[tid] * r.close[t * r.lda + bk[tid]];   // w * price
        }
        __syncthreads();
        if (tid == 0) {
            r.sums[i * 4 + side] = pairwise_dense(sh.x, k);
            double den = 0.0;                                       // builtin sum(): 0 + ...
            for (int a = 0; a < k; ++a) den = den + sh.c[a];
            r.sums[i * 4 + 2 + side] = den;
            if (sh.misc[4]) r.status[i] = 1;
        }
        // union positions of the members vs the previous / next rebalance date
        if (tid < k) {
            const int a = bk[tid];
            const int wa = a >> 6, ba = a & 63;
            for (int q = 0; q < 2; ++q) {
                const int other = q == 0 ? 0 : 2;                   // prev row / next row
                const bool has = (q == 0 ? tp : tn) >= 0 && ((sh.pw[other][wa] >> ba) & 1ull);
                int pos = -1;
                if (has) {
                    pos = 0;
                    for (int wi = 0; wi < wa; ++wi) pos += __popcll(sh.pw[other][wi] | sh.pw[1][wi]);
                    u64 lowm = ba ? ((1ull << ba) - 1ull) : 0ull;
                    pos += __popcll((sh.pw[other][wa] | sh.pw[1][wa]) & lowm);
                }
                r.upos[((i * 2 + side) * 2 + q) * kMaxK + tid] = pos;
            }
        }
        __syncthreads();
    }
    if (tid < 2) {
        const int other = tid == 0 ? 0 : 2;
        int64_t tot = 0;
        for (int wi = 0; wi < nw; ++wi) tot += __popcll(sh.pw[other][wi] | sh.pw[1][wi]);
        r.usize[i * 2 + tid] = tot;
    }
}

// ---- sequential value / turnover recursion (KKT:864-892) ----------------------------------
// The turnover is numpy's pairwise sum over the union-aligned vector |cur - new| (KKT:839), which
// is zero except at the books' members.  Its summation tree is fixed by the union length and
// the members' positions, so turnover_terms_kernel (parallel over dates) compiles it into a
// short stack program; the sequential scan only evaluates term values (they depend on V) and
// runs the program.  Zero slots contribute exact +0.0 (every term is |.| >= 0), so a subtree
// without members is skipped and a node with one non-empty child passes it up unchanged.
constexpr int kMaxTerms = 4 * kMaxK;
constexpr int kMaxProg = 4 * kMaxTerms;
// program tokens: >= 0 : LEAF starting at term index (token & 0xffff), count (token >> 16);
//                 -1   : ADD (pop b, pop a, push a + b)
struct TermBuild {
    int pos[kMaxTerms], side[kMaxTerms], slot[kMaxTerms];
    int prog[kMaxProg];
    int nprog, m;
};

// symbolic numpy pairwise_sum over positions [lo, lo + n) (terms sorted by position)
__device__ int build_pw(TermBuild& tb, int64_t lo, int64_t n, int b, int e) {
    // returns 1 if the subtree holds a term (pushes one value), else 0
    while (b < e && tb.pos[b] < lo) ++b;
    int ee = b;
    while (ee < e && tb.pos[ee] < lo + n) ++ee;
    if (ee == b) return 0;
    if (n <= 128) {
        const int64_t body = n < 8 ? 0 : n - (n % 8);
        for (int q = b; q < ee; ++q) {
            const int64_t off = tb.pos[q] - lo;
            tb.slot[q] = (n < 8) ? 9 : (off < body ? (int)(off % 8) : 8);   // 9 seq, 8 tail
        }
        tb.prog[tb.nprog++] = b | ((ee - b) << 16);
        return 1;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    const int l = build_pw(tb, lo, n2, b, ee);
    const int r = build_pw(tb, lo + n2, n - n2, b, ee);
    if (l && r) tb.prog[tb.nprog++] = -1;
    return l | r;
}

__global__ __launch_bounds__(64) void turnover_terms_kernel(int64_t nd, const int32_t* k_out,
                                                            const int32_t* books,
                                                            const int32_t* upos,
                                                            const int64_t* usize, int32_t* tside,
                                                            int32_t* tslot, int32_t* tprog,
                                                            int32_t* tcount) {
    __shared__ TermBuild tb;
    __shared__ int pos_s[kMaxTerms], side_s[kMaxTerms];
    __shared__ int cnt;
    const int64_t i = blockIdx.x;
    const int tid = threadIdx.x;
    if (tid == 0) cnt = 0;
    __syncthreads();
    const bool active = i > 0 && k_out[i - 1] > 0;   // current_positions.dropna().empty -> 0
    if (active) {
        const int k = k_out[i], kp = k_out[i - 1];
        for (int e = tid; e < 2 * kp; e += 64) {     // previous members predicted today
            const int side = e / kp, q = e % kp;
            const int a = books[((i - 1) * 2 + side) * kMaxK + q];
            const int pz = upos[(((i - 1) * 2 + side) * 2 + 1) * kMaxK + q];
            if (pz < 0) continue;
            int ns = 2;
            for (int s2 = 0; s2 < 2; ++s2)
                for (int q2 = 0; q2 < k; ++q2)
                    if (books[(i * 2 + s2) * kMaxK + q2] == a) ns = s2;
            const int slot = atomicAdd(&cnt, 1);
            pos_s[slot] = pz;
            side_s[slot] = side * 3 + ns;
        }
        for (int e = tid; e < 2 * k; e += 64) {      // today's members predicted yesterday only
            const int side = e / k, q = e % k;
            const int a = books[(i * 2 + side) * kMaxK + q];
            const int pz = upos[((i * 2 + side) * 2 + 0) * kMaxK + q];
            if (pz < 0) continue;
            bool inprev = false;
            for (int s2 = 0; s2 < 2; ++s2)
                for (int q2 = 0; q2 < kp; ++q2)
                    if (books[((i - 1) * 2 + s2) * kMaxK + q2] == a) inprev = true;
            if (inprev) continue;
            const int slot = atomicAdd(&cnt, 1);
            pos_s[slot] = pz;
            side_s[slot] = 2 * 3 + side;
        }
    }
    __syncthreads();
    const int m = cnt;
    for (int e = tid; e < m; e += 64) {              // sort by union position (distinct)
        int r = 0;
        for (int f = 0; f < m; ++f) r += pos_s[f] < pos_s[e];
        tb.pos[r] = pos_s[e];
        tb.side[r] = side_s[e];
    }
    __syncthreads();
    if (tid == 0) {
        tb.nprog = 0;
        if (m > 0) build_pw(tb, 0, usize[i * 2 + 0], 0, m);
        tcount[i * 2 + 0] = active ? m : -1;
        tcount[i * 2 + 1] = tb.nprog;
    }
    __syncthreads();
    for (int e = tid; e < m; e += 64) {
        tside[i * kMaxTerms + e] = tb.side[e];
        tslot[i * kMaxTerms + e] = tb.slot[e];
    }
    for (int e = tid; e < tb.nprog; e += 64) tprog[i * kMaxProg + e] = tb.prog[e];
}

struct ScanBuf {
    int side[kMaxTerms], slot[kMaxTerms], prog[kMaxProg];
    double sums[4], sums_prev[4];
    int m, nprog;
};

__global__ __launch_bounds__(128) void pnl_scan_kernel(int64_t nd, const double* sums,
                                                      const int32_t* tside, const int32_t* tslot,
                                                      const int32_t* tprog,
                                                      const int32_t* tcount, double v0,
                                                      double rate, double* value,
                                                      double* turnover, double* long_ret,
                                                      double* short_ret) {
    __shared__ ScanBuf buf[2];
    __shared__ double val[kMaxTerms];
    __shared__ double stk[kMaxTerms + 1];
    __shared__ double Vs, Vprev;
    const int tid = threadIdx.x;
    // wave 1 (threads 64..127) stages date i+1 while lane 0 of wave 0 runs date i's program
    auto load = [&](int64_t i, ScanBuf& B) {
        const int lt = tid - 64;
        const int m = tcount[i * 2 + 0], np = tcount[i * 2 + 1];
        for (int e = lt; e < m; e += 64) {
            B.side[e] = tside[i * kMaxTerms + e];
            B.slot[e] = tslot[i * kMaxTerms + e];
        }
        for (int e = lt; e < np; e += 64) B.prog[e] = tprog[i * kMaxProg + e];
        if (lt < 4) {
            B.sums[lt] = sums[i * 4 + lt];
            B.sums_prev[lt] = i > 0 ? sums[(i - 1) * 4 + lt] : 0.0;
        }
        if (lt == 0) { B.m = m; B.nprog = np; }
    };
    if (tid == 0) { Vs = v0; Vprev = v0; value[0] = v0; }
    if (tid >= 64) load(0, buf[0]);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    for (int64_t i = 0; i < nd; ++i) {
        ScanBuf& B = buf[i & 1];
        const double V = Vs, Vp = Vprev;
        const int m = B.m;
        if (m > 0) {                                  // term values |c - n| (KKT:881-882, 839)
            const double sizep = Vp / 2, size = V / 2;
            for (int e = tid; e < m; e += 128) {
                const int sd = B.side[e];
                const int ps = sd / 3, ns = sd % 3;
                const double c = ps == 0 ? sizep / B.sums_prev[2]
                                         : (ps == 1 ? -sizep / B.sums_prev[3] : 0.0);
                const double nv = ns == 0 ? size / B.sums[2] : (ns == 1 ? -size / B.sums[3] : 0.0);
                const double d = c - nv;
                val[e] = d < 0 ? -d : d;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (tid == 0) {
            double to = 0.0;
            if (m > 0) {
                int sp = 0;
                for (int q = 0; q < B.nprog; ++q) {
                    const int tk = B.prog[q];
                    if (tk < 0) {
                        const double bb = stk[--sp];
                        const double aa = stk[--sp];
                        stk[sp++] = aa + bb;
                        continue;
                    }
                    const int t0 = tk & 0xffff, cnt = tk >> 16;
                    double res;
                    if (B.slot[t0] == 9) {            // leaf shorter than 8: sequential from 0
                        res = 0.;
                        for (int e = t0; e < t0 + cnt; ++e) res += val[e];
                    } else {                          // 8 accumulators, then the tail
                        double r[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                        for (int e = t0; e < t0 + cnt; ++e)
                            if (B.slot[e] < 8) r[B.slot[e]] += val[e];
                        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
                        for (int e = t0; e < t0 + cnt; ++e)
                            if (B.slot[e] == 8) res += val[e];
                    }
                    stk[sp++] = res;
                }
                to = stk[0] / 2;
            }
            double daily = (B.sums[0] - B.sums[1]) / 2;
            long_ret[i] = B.sums[0];
            short_ret[i] = B.sums[1];
            turnover[i] = to;
            daily -= (to * rate) / V;
            const double Vn = V * (1 + daily);
            value[i + 1] = Vn;
            Vprev = V;
            Vs = Vn;
        } else if (tid >= 64 && i + 1 < nd) {
            load(i + 1, buf[(i + 1) & 1]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
}

}  // namespace
}  // namespace afm

using namespace afm;

extern "C" int afm_rebalance_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda,
                                 const int32_t* dates, int64_t nd, const double* pred,
                                 const uint64_t* trad_bits, const double* hist,
                                 const uint64_t* hist_bits, int64_t h_t0, int64_t h_t1,
                                 int64_t window, const double* close, const double* tmr,
                                 int top_n, double lo, double hi, int32_t* k_out,
                                 int32_t* books, double* weights, double* sums, int32_t* upos,
                                 int64_t* usize, int32_t* status) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(T > 0 && A > 0 && lda >= A && lda % 64 == 0, "bad panel shape");
    AFM_CHECK_ARG((A + 63) / 64 <= kMaxWords, "too many assets (max 32768)");
    AFM_CHECK_ARG(top_n >= 0 && top_n <= kMaxK, "top_n must be in [0, 64]");
    AFM_CHECK_ARG(dates && pred && trad_bits && hist && hist_bits && close && tmr && k_out &&
                      books && weights && sums && upos && usize && status, "null buffer");
    AFM_CHECK_ARG(lo <= hi, "lo > hi");
    if (nd <= 0) return AFM_OK;
    RebArgs r{T, lda, A, dates, nd, pred, trad_bits, hist, hist_bits, h_t0, h_t1, window, close,
              tmr, top_n, lo, hi, k_out, books, weights, sums, upos, usize, status};
    const size_t smem = sizeof(Shared);
    AFM_HIP(hipFuncSetAttribute((const void*)rebalance_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
    hipLaunchKernelGGL(rebalance_kernel, dim3((unsigned)nd), dim3(kT), smem, ctx->stream, r);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_pnl_scan_f64(afm_ctx* ctx, int64_t nd, const int32_t* k_out,
                                const int32_t* books, const double* sums, const int32_t* upos,
                                const int64_t* usize, double v0, double rate, double* value,
                                double* turnover, double* long_ret, double* short_ret) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(k_out && books && sums && upos && usize && value && turnover && long_ret &&
                      short_ret, "null buffer");
    if (nd <= 0) return AFM_OK;
    int32_t* work = nullptr;
    const size_t words = (size_t)nd * (2 * kMaxTerms + kMaxProg + 2);
    AFM_HIP(hipMallocAsync((void**)&work, sizeof(int32_t) * words, ctx->stream));
    int32_t* tside = work;
    int32_t* tslot = work + nd * kMaxTerms;
    int32_t* tprog = work + 2 * nd * kMaxTerms;
    int32_t* tcount = tprog + nd * kMaxProg;
    hipLaunchKernelGGL(turnover_terms_kernel, dim3((unsigned)nd), dim3(64), 0, ctx->stream, nd,
                       k_out, books, upos, usize, tside, tslot, tprog, tcount);
    AFM_HIP(hipGetLastError());
    hipLaunchKernelGGL(pnl_scan_kernel, dim3(1), dim3(128), 0, ctx->stream, nd, sums, tside, tslot,
                       tprog, tcount, v0, rate, value, turnover, long_ret, short_ret);
    AFM_HIP(hipGetLastError());
    AFM_HIP(hipFreeAsync(work, ctx->stream));
    return AFM_OK;
}

extern "C" int afm_min_variance_weights_f64(afm_ctx* ctx, const double* R, int64_t rows,
                                            int64_t ld, int k, double lo, double hi, double* w,
                                            double* cov, int32_t* status) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(k >= 1 && k <= kMaxK && ld >= k && rows >= 0, "need 1 <= k <= 64, ld >= k");
    AFM_CHECK_ARG(R && w && cov && status && lo <= hi, "bad arguments");
    const size_t smem = sizeof(Shared);
    AFM_HIP(hipFuncSetAttribute((const void*)weights_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
    hipLaunchKernelGGL(weights_kernel, dim3(1), dim3(kT), smem, ctx->stream, R, rows, ld, k, lo,
                       hi, w, cov, status);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

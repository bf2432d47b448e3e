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

#include <algorithm>
#include <type_traits>
#include <vector>

#pragma clang fp contract(off)

namespace afm {
namespace {

typedef unsigned long long u64;
constexpr int kT = 256;        // threads per workgroup
constexpr int kMaxK = 128;     // book-size cap; the global book arrays are [nd][2][kMaxK]
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
    double* hscr;             // scratch [nd][2][top_n][hrows]: books' history windows (or null)
    const double* histT;      // books over 32 names: [lda][hTn] history, member-major, NaN absent
    int64_t hT0, hTn;         // its date range [hT0, hT0 + hTn)
    int64_t hrows;            // rows per window: window, or h_t1 - h_t0
    int probe;                // experiments (AFM_REB_PROBE): 1 skip the QP, 2 skip the covariance,
    int64_t* stamps;          // 4 phase timestamps per workgroup ([nd][2][5])
    // outputs (per rebalance date i)
    int32_t* k_out;           // [nd]
    int32_t* books;           // [nd][2][kMaxK] asset indices (long book, short book)
    double* weights;          // [nd][2][kMaxK]
    double* sums;             // [nd][4]: long_ret, short_ret, den_long, den_short
    int32_t* upos;            // [nd][2][2][kMaxK]: union position vs prev / vs next (-1 absent)
    int64_t* usize;           // [nd][2]: |P_prev U P_i|, |P_i U P_next|
    int32_t* status;          // [nd] (zeroed by the launcher): |1 QP iteration cap, 2 k > cap
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

__device__ __forceinline__ void lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// packed symmetric index of the member pair (a, b)
__device__ __forceinline__ int tri(int a, int b) {
    return a >= b ? a * (a + 1) / 2 + b : b * (b + 1) / 2 + a;
}

// LDS of one (date, book) workgroup, sized for books of at most KM names: the covariance S
// (packed, tri()), and a union of the history staging of the covariance phase, the Cholesky
// factor of the QP or the tie buffer of the selection.  The factor is packed by member PAIR: the
// entry of {q, q'} belongs to whichever of the two was factored later (row) -- one orientation
// per pair -- so members can leave and join the factor order without moving data.
// LDS of the workgroup QP (qp_block): broadcast vectors, the two column halves' partial
// products and the reduction slots
struct QpLds {
    double pubk[2][4][128];              // published rows of M (block sweep: 4, double-buffered)
    double vc[128], vw[128], vu[128];    // broadcast vectors: S_FB w_B, w, u~
    double part[4][2][128];              // [product][column half][row]
    double red[6][4][4];                 // [use][wave][value]
    int code[4];
};

template <int KM>
struct Shared {
    u64 pw[3][kMaxWords];                // prediction presence rows: prev, cur, next
    int hist[256];
    int scan[kT];
    int misc[8];
    u64 keysel[KM];
    int idxsel[KM];
    int book[KM];
    int ord[KM], state[KM];              // QP: factor order (members), bound state per member
    double w[KM], x[KM], c[KM];
    double sinv[258];                    // 1 / n for the Welford updates (n <= 257)
    double S[KM * (KM + 1) / 2];
    u64 pm[KM > 32 ? KM : 1];            // presence words of the staged chunk (MFMA covariance)
    union {
        double hv[KM][65];               // staged history chunk [member][date]
        double L[KM * (KM + 1) / 2];     // Cholesky factor of S_FF (packed by member pair)
        // the workgroup QP of books of more than 32 names (absent from the 32-name layout, whose
        // LDS size sets how many headline workgroups share a CU)
        typename std::conditional<(KM > 32), QpLds, char>::type qp;
    } u;
};

static_assert(sizeof(Shared<kMaxK>) <= 160 * 1024, "rebalance LDS over the CU's 160 KB");
static_assert(sizeof(Shared<32>) <= 40 * 1024, "headline rebalance LDS: 4 workgroups per CU");

// Welford pairwise-complete covariance (pandas nancorr(cov=True), KKT:821-822: rows in date
// order, a pair's rows where both values are finite) of the k members' history rows [0, rows)
// into sh.S.  Rows are staged through LDS 64 at a time (get(m, row): value or NaN), every
// thread issuing its loads of a chunk back to back; one thread per member pair.
template <int KM, class Get>
__device__ __forceinline__ void book_cov(Shared<KM>& sh, const int k, const int64_t rows,
                                         Get get) {
    const int tid = threadIdx.x;
    constexpr int EPT = KM * 64 / kT;                // staged values per thread
    for (int e = tid; e <= 257; e += kT) sh.sinv[e] = e ? 1. / (double)e : 0.0;
    const bool table = rows <= 256;                  // nobs + 1 <= 257
    const int npairs = k * (k + 1) / 2;
    constexpr int P = KM >= 64 ? 4 : 1;              // member pairs per thread and pass
    for (int pb = 0; pb < npairs; pb += P * kT) {
        int pi[P], pj[P], nobs[P];
        double mx[P], my[P], cxy[P], invn[P];
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const int pq = pb + p * kT + tid;
            int a = 0, q = pq < npairs ? pq : 0;     // pq -> (xi >= yi), row-major lower triangle
            while (q > a) { q -= a + 1; ++a; }
            pi[p] = a;
            pj[p] = q;
            nobs[p] = 0;
            invn[p] = 1.0;
            mx[p] = 0;
            my[p] = 0;
            cxy[p] = 0;
        }
        for (int64_t h0 = 0; h0 < rows; h0 += 64) {
            double v[EPT];
#pragma unroll
            for (int j = 0; j < EPT; ++j) {
                const int e = tid + j * kT;
                v[j] = e < k * 64 ? get(e >> 6, h0 + (e & 63)) : 0.0;
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < EPT; ++j) {
                const int e = tid + j * kT;
                if (e < k * 64) sh.u.hv[e >> 6][e & 63] = v[j];
            }
            __syncthreads();
            const int nd = (int)((rows - h0) < 64 ? (rows - h0) : 64);
            // P independent Welford chains, branch-free; 1 / (nobs + 1) comes from the table,
            // fetched one date ahead (or divided when the window exceeds the table)
            for (int d = 0; d < nd; ++d) {
                double vx[P], vy[P];
#pragma unroll
                for (int p = 0; p < P; ++p) {
                    vx[p] = sh.u.hv[pi[p]][d];
                    vy[p] = sh.u.hv[pj[p]][d];
                }
#pragma unroll
                for (int p = 0; p < P; ++p) {
                    const bool f = __builtin_isfinite(vx[p]) && __builtin_isfinite(vy[p]);
                    const double inv = table ? invn[p] : 1. / (double)(nobs[p] + 1);
                    const double dx = vx[p] - mx[p], dy = vy[p] - my[p];
                    const double mxn = mx[p] + inv * dx;
                    const double myn = my[p] + inv * dy;
                    const double cn = cxy[p] + (vx[p] - mxn) * dy;
                    nobs[p] += f ? 1 : 0;
                    mx[p] = f ? mxn : mx[p];
                    my[p] = f ? myn : my[p];
                    cxy[p] = f ? cn : cxy[p];
                    if (table) invn[p] = sh.sinv[nobs[p] + 1];
                }
            }
        }
#pragma unroll
        for (int p = 0; p < P; ++p) {
            if (pb + p * kT + tid < npairs) {
                double cv = __builtin_nan("");
                if (nobs[p] >= 2) cv = cxy[p] / ((double)nobs[p] - 1.0);
                sh.S[tri(pi[p], pj[p])] = cv;
            }
        }
    }
    __syncthreads();
}

// ---- pairwise-complete covariance on fp64 MFMA (books of more than 32 names) -----------------
// The same statistic as book_cov (pandas nancorr(cov=True): per pair, the rows where both values
// are finite) written as masked SYRKs over the window.  With m the presence mask, c_m a centring
// constant per member and x~ = m * (x - c_m):
//   N = M M',  C = X~ X~',  P = X~ M',  Q = M X~'     (P_ij = sum over both-present rows of x~_i,
//   Q_ij = the same of x~_j), cov_ij = (C_ij - P_ij Q_ij / N_ij) / (N_ij - 1), NaN for N_ij < 2.
// C, P and Q are v_mfma_f64_16x16x4_f64 on 16-member tiles (the window rows are the k dim): 36
// tile pairs (I <= J) of at most 8 tiles, pair q on wave q % 4, 27 accumulators per wave, ONE pass
// over the window; N is counted on the VALU from the staged chunk's presence words (popcount of
// m_i & m_j per 64 rows).  c_m is the member's first finite value in the window's first 64 rows
// (shifted data: the cancellation in C - PQ/N is then O(1) in the variance, rel ~1e-15 of S on
// the test books, vs 1e-12 for the bar of tests/test_portfolio_gpu.py).
typedef double d4 __attribute__((ext_vector_type(4)));

struct CovPairs {
    int I[36], J[36];
    constexpr CovPairs() : I(), J() {
        int q = 0;
        for (int j = 0; j < 8; ++j)
            for (int i = 0; i <= j; ++i) { I[q] = i; J[q] = j; ++q; }
    }
};

template <int KM, int W, class Get>
__device__ __noinline__ void cov_mfma_wave(Shared<KM>& sh, const int k, const int64_t rows,
                                           Get get) {
    static_assert(KM == 128, "MFMA covariance: 8 tiles of 16 members");
    constexpr CovPairs tab{};
    constexpr int NS = 9;                            // slots: pair q = W + 4 s
    const int tid = threadIdx.x, lane = tid & 63;
    const int fi = lane & 15, kk = lane >> 4;
    const int nt = (k + 15) / 16;
    double mu[8];
    d4 c[NS], pp[NS], qq[NS];
    int nn[NS][4];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        c[s] = d4{0.0, 0.0, 0.0, 0.0};
        pp[s] = c[s];
        qq[s] = c[s];
#pragma unroll
        for (int r = 0; r < 4; ++r) nn[s][r] = 0;
    }
    // software-pipelined staging: chunk c + 1 is loaded into registers while chunk c is multiplied
    constexpr int EPT = KM * 64 / kT;
    double v[EPT];
    auto load = [&](int64_t h0) {                  // branch-free: every load in flight at once
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const int e = tid + j * kT;
            const int m = (e >> 6) < k ? (e >> 6) : k - 1;
            const double x = get(m, h0 + (e & 63));
            v[j] = e < k * 64 ? x : 0.0;
        }
    };
    if (rows > 0) load(0);
    for (int64_t h0 = 0; h0 < rows; h0 += 64) {
        __syncthreads();                             // the previous chunk's readers are done
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const int e = tid + j * kT;              // member e >> 6 (uniform per wave), row lane
            const u64 mk = __ballot(e < k * 64 && __builtin_isfinite(v[j]));
            if (e < k * 64) sh.u.hv[e >> 6][e & 63] = v[j];
            if (lane == 0 && e < k * 64) sh.pm[e >> 6] = mk;
        }
        __syncthreads();
        if (h0 + 64 < rows) load(h0 + 64);
        if (h0 == 0) {                               // centring constants
            if (tid < k) {
                double c0 = 0.0;
                for (int d = 0; d < 64; ++d) {
                    const double v = sh.u.hv[tid][d];
                    if (__builtin_isfinite(v)) { c0 = v; break; }
                }
                sh.x[tid] = c0;
            }
            __syncthreads();
#pragma unroll
            for (int t = 0; t < 8; ++t) mu[t] = 16 * t + fi < k ? sh.x[16 * t + fi] : 0.0;
        }
        // N: both-present counts of this chunk's rows, element (16 I + kk + 4 r, 16 J + fi)
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int q = W + 4 * s;
            if (q < 36 && tab.J[q] < nt) {
                const u64 mj = sh.pm[16 * tab.J[q] + fi];
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    nn[s][r] += __popcll(mj & sh.pm[16 * tab.I[q] + kk + 4 * r]);
            }
        }
        const int nks = (int)((rows - h0) < 64 ? (rows - h0 + 3) / 4 : 16);
        for (int it = 0; it < nks; ++it) {
            double x[8], m[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int mem = 16 * t + fi, row = 4 * it + kk;
                const double v = sh.u.hv[mem][row];
                const bool f = mem < k && h0 + row < rows && __builtin_isfinite(v);
                x[t] = f ? v - mu[t] : 0.0;
                m[t] = f ? 1.0 : 0.0;
            }
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const int q = W + 4 * s;
                if (q < 36 && tab.J[q] < nt) {
                    const int I = tab.I[q], J = tab.J[q];
                    c[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(x[I], x[J], c[s], 0, 0, 0);
                    pp[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(x[I], m[J], pp[s], 0, 0, 0);
                    qq[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(m[I], x[J], qq[s], 0, 0, 0);
                }
            }
        }
    }
    // element (i, j), i >= j (one lane each)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int q = W + 4 * s;
        if (q < 36 && tab.J[q] < nt) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * tab.I[q] + kk + 4 * r, j = 16 * tab.J[q] + fi;
                if (i < k && j < k && (tab.I[q] < tab.J[q] || i >= j)) {
                    const double n = (double)nn[s][r];
                    sh.S[tri(i, j)] = nn[s][r] >= 2 ? (c[s][r] - pp[s][r] * qq[s][r] / n) /
                                                          (n - 1.0)
                                                    : __builtin_nan("");
                }
            }
        }
    }
}

template <int KM, class Get>
__device__ __forceinline__ void book_cov_mfma(Shared<KM>& sh, const int k, const int64_t rows,
                                              Get get) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    switch (wave) {
        case 0: cov_mfma_wave<KM, 0>(sh, k, rows, get); break;
        case 1: cov_mfma_wave<KM, 1>(sh, k, rows, get); break;
        case 2: cov_mfma_wave<KM, 2>(sh, k, rows, get); break;
        default: cov_mfma_wave<KM, 3>(sh, k, rows, get); break;
    }
    __syncthreads();
}

// k largest keys among candidates (key valid when cand), ties -> smaller index first.
// Writes the selected indices, sorted (key desc, index asc), to out[0..k).
template <int KM>
__device__ __forceinline__ void select_top(const RebArgs& r, Shared<KM>& sh, int64_t t, int k,
                                           bool largest, int* out) {
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

// Radix digit choice of select_top_reg, on wave 0: the largest digit d whose suffix count
// sum_{d' >= d} hist[d'] reaches `need` -> misc[0] = d, misc[1] = need - (count above d),
// misc[2] = hist[d].  Lane l owns digits 4l..4l+3; a shuffle suffix scan replaces the serial
// 256-step loop.
template <int KM>
__device__ __forceinline__ void digit_pick(Shared<KM>& sh, const int need) {
    const int tid = threadIdx.x;
    if (tid >= 64) return;
    const int h0 = sh.hist[4 * tid], h1 = sh.hist[4 * tid + 1], h2 = sh.hist[4 * tid + 2],
              h3 = sh.hist[4 * tid + 3];
    const int s = h0 + h1 + h2 + h3;
    int S = s;                                       // inclusive suffix sum over lanes
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_down(S, o, 64);
        if (tid + o < 64) S += v;
    }
    const u64 m = __ballot(S >= need);
    const int L = 63 - __clzll(m);
    if (tid == L) {
        int acc = S - s, d = 4 * L, hd = h0;
        if (acc + h3 >= need) { d = 4 * L + 3; hd = h3; }
        else if (acc + h3 + h2 >= need) { d = 4 * L + 2; hd = h2; acc += h3; }
        else if (acc + h3 + h2 + h1 >= need) { d = 4 * L + 1; hd = h1; acc += h3 + h2; }
        else acc += h3 + h2 + h1;
        sh.misc[0] = d;
        sh.misc[1] = need - acc;
        sh.misc[2] = hd;
    }
}

// select_top on register-resident keys: ks[j] = okey of asset j * kT + tid (0: not a candidate).
// Same result as select_top (threshold by exact radix select; ties at the threshold taken by
// ascending index), without re-reading the predictions for every digit.
template <int KR, int KM>
__device__ __forceinline__ bool select_top_reg(Shared<KM>& sh, const u64 (&ks)[KR], int k,
                                               bool largest, int* out) {
    const int tid = threadIdx.x;
    u64 prefix = 0, pmask = 0;
    int need = k, eqtot = 0;
    for (int shift = 56; shift >= 0; shift -= 8) {
        sh.hist[tid] = 0;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < KR; ++j) {
            if (ks[j] != 0ull) {
                const u64 kk = largest ? ks[j] : ~ks[j];
                if ((kk & pmask) == prefix) atomicAdd(&sh.hist[(kk >> shift) & 255], 1);
            }
        }
        __syncthreads();
        digit_pick(sh, need);
        __syncthreads();
        prefix |= (u64)sh.misc[0] << shift;
        pmask |= 255ull << shift;
        need = sh.misc[1];
        eqtot = sh.misc[2];
        __syncthreads();
    }
    // keys > tau are all taken; of the eqtot keys == tau the `need` smallest indices (a tie
    // straddling the threshold is rare: its indices are ranked by counting in LDS)
    int* eqbuf = reinterpret_cast<int*>(&sh.u);
    constexpr int kEqMax = (int)(sizeof(sh.u) / sizeof(int));
    const bool all_eq = eqtot == need;
    if (!all_eq && eqtot > kEqMax) return false;     // (uniform) caller takes the global path
    if (tid == 0) { sh.misc[3] = 0; sh.misc[6] = 0; }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < KR; ++j) {
        if (ks[j] != 0ull) {
            const u64 kk = largest ? ks[j] : ~ks[j];
            if (kk > prefix || (all_eq && kk == prefix)) {
                const int pos = atomicAdd(&sh.misc[3], 1);
                sh.keysel[pos] = kk;
                sh.idxsel[pos] = j * kT + tid;
            } else if (kk == prefix) {
                const int pos = atomicAdd(&sh.misc[6], 1);
                if (pos < kEqMax) eqbuf[pos] = j * kT + tid;
            }
        }
    }
    __syncthreads();
    if (!all_eq) {
        const int ngt = sh.misc[3];
        const int neq = sh.misc[6];                  // == eqtot <= kEqMax
        for (int e = tid; e < neq; e += kT) {
            const int me = eqbuf[e];
            int rank = 0;
            for (int f = 0; f < neq; ++f) rank += eqbuf[f] < me;
            if (rank < need) {
                sh.keysel[ngt + rank] = prefix;
                sh.idxsel[ngt + rank] = me;
            }
        }
    }
    __syncthreads();
    if (tid < k) {
        const u64 mk = sh.keysel[tid];
        const int mi = sh.idxsel[tid];
        int rank = 0;
        for (int j = 0; j < k; ++j) {
            const u64 ok = sh.keysel[j];
            const int oi = sh.idxsel[j];
            rank += (ok > mk) || (ok == mk && oi < mi);
        }
        out[rank] = mi;
    }
    __syncthreads();
    return true;
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

// ---- wave-level helpers of the QP (wave 0 runs it alone: no workgroup barrier inside) --------
__device__ __forceinline__ double wave_sum(double v) {       // butterfly: identical in all lanes
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// lexicographic (v, code) minimum over the wave, in every lane
__device__ __forceinline__ void wave_argmin(double& v, int& code) {
    for (int o = 32; o >= 1; o >>= 1) {
        const double v2 = __shfl_xor(v, o, 64);
        const int c2 = __shfl_xor(code, o, 64);
        if (v2 < v || (v2 == v && c2 < code)) { v = v2; code = c2; }
    }
}

__device__ __forceinline__ double rdlane(double v, int l) {   // l uniform
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// min w'Sw  s.t. sum w = 1, lo <= w <= hi for the k x k covariance sh.S -> sh.w, by the primal
// active-set method of oracle/portfolio.py:box_qp_weights (KKT:811-833 solved exactly).  Each
// step solves [S_FF 1; 1' 0][w_F; lam] = [-S_FB w_B; b] with M = S_FF^-1 kept EXPLICITLY and
// updated as the free set F changes: a member bound by the ratio test leaves by the rank-1
// deflation M <- M - m_j m_j' / M_jj, a member released by its multiplier joins by bordering
// (u = M s, d = S_jj - s'u, M <- M + u u'/d).  Every step is then a handful of lane-parallel
// matrix-vector products and rank-1 updates -- no sequential substitution chain.  The optimum is
// unique (S positive definite), so only the end point, not the path, is compared with the
// oracle's refactor-every-step solve (rel 1e-9).
//
// qp_setup (every thread of the block): the start point w = 1/k, all members free, and
// M = S^-1 by the sweep operator over all k members, each pivot's update spread over the block.
// Returns false (uniform) when S is not finite: weights NaN, iteration cap reported.
template <int KM>
__device__ __forceinline__ bool qp_setup(Shared<KM>& sh, const int n) {
    const int tid = threadIdx.x;
    const int np = n * (n + 1) / 2;
    int bad = 0;
    for (int e = tid; e < np; e += kT) bad |= !__builtin_isfinite(sh.S[e]);
    if (__syncthreads_or(bad)) {
        for (int q = tid; q < n; q += kT) sh.w[q] = __builtin_nan("");
        __syncthreads();
        return false;
    }
    for (int q = tid; q < n; q += kT) {
        sh.w[q] = 1.0 / n;
        sh.state[q] = 0;
        sh.ord[q] = q;
    }
    // sweep(k): A_ij -= A_ik A_jk / A_kk (i, j != k); A_ik /= A_kk; A_kk = -1 / A_kk.  After every
    // member is swept, A = -S^-1.  The packed elements stay in registers (EPT per thread); each
    // pivot publishes its column through LDS (double-buffered: one barrier per pivot).
    constexpr int EPT = (KM * (KM + 1) / 2 + kT - 1) / kT;
    double av[EPT];
    int ij[EPT];
#pragma unroll
    for (int m = 0; m < EPT; ++m) {
        const int e = tid + m * kT;
        int i = (int)((__builtin_sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
        if (i * (i + 1) / 2 > e) --i;
        if ((i + 1) * (i + 2) / 2 <= e) ++i;
        ij[m] = (i << 16) | (e - i * (i + 1) / 2);
        av[m] = e < np ? sh.S[e] : 0.0;
    }
    for (int k = 0; k < n; ++k) {
        double* colk = (k & 1) ? sh.x : sh.c;
#pragma unroll
        for (int m = 0; m < EPT; ++m) {
            const int i = ij[m] >> 16, j = ij[m] & 0xffff;
            if (tid + m * kT < np) {
                if (j == k) colk[i] = av[m];
                else if (i == k) colk[j] = av[m];
            }
        }
        __syncthreads();
        const double rd = 1.0 / colk[k];
#pragma unroll
        for (int m = 0; m < EPT; ++m) {
            const int i = ij[m] >> 16, j = ij[m] & 0xffff;
            if (tid + m * kT < np) {
                if (i != k && j != k) av[m] -= colk[i] * colk[j] * rd;
                else if (i == k && j == k) av[m] = -rd;
                else av[m] = av[m] * rd;
            }
        }
    }
#pragma unroll
    for (int m = 0; m < EPT; ++m)
        if (tid + m * kT < np) sh.u.L[tid + m * kT] = -av[m];   // M = S^-1
    __syncthreads();
    return true;
}

// The iterations, on wave 0 alone (no workgroup barrier inside): lanes own free-list
// positions a = lane + 64 r (sh.ord[a] = member).  Returns true if the iteration cap was hit
// (uniform in wave 0).
template <int KM>
__device__ __forceinline__ bool qp_wave(Shared<KM>& sh, const int n, const double lo,
                                        const double hi) {
    constexpr int R = (KM + 63) / 64;
    const int lane = threadIdx.x & 63;
    double* M = sh.u.L;
    int* blist = sh.idxsel;                            // bound members (selection is done)
    int nf = n;
    bool capped = false;
    const int max_it = 4 * n + 8;
    for (int it = 0; it < max_it; ++it) {
        if (nf == 0) break;
        if (it == max_it - 1) capped = true;
        int oq[R];
        double bs = 0.0;
        int nb = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int p = lane + 64 * r;                // as a member index: bound list + sum
            const bool isb = p < n && sh.state[p] != 0;
            if (isb) bs += sh.w[p];
            const u64 m = __ballot(isb);
            if (isb) blist[nb + __popcll(m & ((1ull << lane) - 1ull))] = p;
            nb += __popcll(m);
            oq[r] = p < nf ? sh.ord[p] : 0;             // as a free-list position
        }
        const double bfree = 1.0 - wave_sum(bs);
        lds_sync();
        double cpos[R];                                // c = S_FB w_B, by free position
#pragma unroll
        for (int r = 0; r < R; ++r) {
            double cc = 0.0;
            if (lane + 64 * r < nf) {
#pragma unroll 4
                for (int i = 0; i < nb; ++i) {
                    const int q = blist[i];
                    cc = cc + sh.S[tri(q, oq[r])] * sh.w[q];
                }
            }
            cpos[r] = cc;
        }
        // y1 = M 1, y2 = M c over the free set; position b's member and c_b by v_readlane
        double y1[R], y2[R];
#pragma unroll
        for (int r = 0; r < R; ++r) { y1[r] = 0.0; y2[r] = 0.0; }
#pragma unroll
        for (int rb = 0; rb < R; ++rb) {
            const int lim = nf - 64 * rb < 64 ? nf - 64 * rb : 64;
#pragma unroll 4
            for (int lb = 0; lb < lim; ++lb) {
                const int qb = __builtin_amdgcn_readlane(oq[rb], lb);
                const double cb = rdlane(cpos[rb], lb);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (lane + 64 * r < nf) {
                        const double mab = M[tri(oq[r], qb)];
                        y1[r] = y1[r] + mab;
                        y2[r] = y2[r] + mab * cb;
                    }
                }
            }
        }
        double s1 = 0.0, s2 = 0.0;
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (lane + 64 * r < nf) { s1 += y1[r]; s2 += y2[r]; }
        s1 = wave_sum(s1);
        s2 = wave_sum(s2);
        const double lam = -(bfree + s2) / s1;
        double x[R];
        bool infeas = false;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            x[r] = -y2[r] - lam * y1[r];
            if (lane + 64 * r < nf && (!(x[r] >= lo) || !(x[r] <= hi))) infeas = true;
        }
        if (!__ballot(infeas)) {
            // feasible: take x; release the bound member with the most negative multiplier
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (lane + 64 * r < nf) sh.w[oq[r]] = x[r];
            lds_sync();
            double vmin = __builtin_inf();
            int qmin = 0x7fffffff;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int q = lane + 64 * r;
                if (q < n && sh.state[q] != 0) {
                    double g = 0.0;
#pragma unroll 4
                    for (int b = 0; b < n; ++b) g = g + sh.S[tri(q, b)] * sh.w[b];
                    g = g + lam;
                    const double v = sh.state[q] < 0 ? g : -g;
                    if (v < vmin) { vmin = v; qmin = q; }
                }
            }
            wave_argmin(vmin, qmin);
            if (!(vmin < 0.0)) break;
            // bordering: u = M s (s = S[F][qmin]), d = S_jj - s'u
            const int j = qmin;
            double sv[R], u[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                sv[r] = lane + 64 * r < nf ? sh.S[tri(oq[r], j)] : 0.0;
                u[r] = 0.0;
            }
#pragma unroll
            for (int rb = 0; rb < R; ++rb) {
                const int lim = nf - 64 * rb < 64 ? nf - 64 * rb : 64;
#pragma unroll 4
                for (int lb = 0; lb < lim; ++lb) {
                    const int qb = __builtin_amdgcn_readlane(oq[rb], lb);
                    const double sb = rdlane(sv[rb], lb);
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        if (lane + 64 * r < nf) u[r] = u[r] + M[tri(oq[r], qb)] * sb;
                }
            }
            double su = 0.0;
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (lane + 64 * r < nf) su += sv[r] * u[r];
            const double d = sh.S[tri(j, j)] - wave_sum(su);
            const double rd = 1.0 / d;
            double ua[R];
#pragma unroll
            for (int r = 0; r < R; ++r) ua[r] = u[r] * rd;
#pragma unroll
            for (int rb = 0; rb < R; ++rb) {
                const int lim = nf - 64 * rb < 64 ? nf - 64 * rb : 64;
#pragma unroll 4
                for (int lb = 0; lb < lim; ++lb) {
                    const int b = 64 * rb + lb;
                    const int qb = __builtin_amdgcn_readlane(oq[rb], lb);
                    const double ub = rdlane(u[rb], lb);
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        if (lane + 64 * r < nf && lane + 64 * r >= b) {
                            const int e = tri(oq[r], qb);
                            M[e] = M[e] + ua[r] * ub;
                        }
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (lane + 64 * r < nf) M[tri(oq[r], j)] = -ua[r];
            if (lane == 0) {
                M[tri(j, j)] = rd;
                sh.ord[nf] = j;
                sh.state[j] = 0;
            }
            lds_sync();
            ++nf;
        } else {
            // ratio test: the first member (ascending index) to hit its bound along x - w
            double amin = __builtin_inf();
            int code = 0x7fffffff;                     // 2 * member + (bound is hi)
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (lane + 64 * r < nf) {
                    const int q = oq[r];
                    const double wq = sh.w[q];
                    const double pq = x[r] - wq;
                    if (x[r] < lo && pq < 0) {
                        const double al = (lo - wq) / pq;
                        if (al < 1.0 && (al < amin || (al == amin && 2 * q < code))) {
                            amin = al;
                            code = 2 * q;
                        }
                    } else if (x[r] > hi && pq > 0) {
                        const double al = (hi - wq) / pq;
                        if (al < 1.0 && (al < amin || (al == amin && 2 * q + 1 < code))) {
                            amin = al;
                            code = 2 * q + 1;
                        }
                    }
                }
            }
            wave_argmin(amin, code);
            const bool hit = code != 0x7fffffff;
            const double alpha = hit ? amin : 1.0;
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (lane + 64 * r < nf) {
                    const double wq = sh.w[oq[r]];
                    sh.w[oq[r]] = wq + alpha * (x[r] - wq);
                }
            lds_sync();
            if (hit) {
                const int jb = code >> 1;
                if (lane == 0) {
                    sh.w[jb] = (code & 1) ? hi : lo;
                    sh.state[jb] = (code & 1) ? 1 : -1;
                }
                // deflation M <- M - m m' / m_jj over F \ {jb}, m = M[F][jb]
                int pj = 0;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const u64 m = __ballot(lane + 64 * r < nf && oq[r] == jb);
                    if (m) pj = 64 * r + __builtin_ctzll(m);
                }
                const double rjj = 1.0 / M[tri(jb, jb)];
                double mj[R], ma[R];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    mj[r] = lane + 64 * r < nf ? M[tri(oq[r], jb)] : 0.0;
                    ma[r] = mj[r] * rjj;
                }
#pragma unroll
                for (int rb = 0; rb < R; ++rb) {
                    const int lim = nf - 64 * rb < 64 ? nf - 64 * rb : 64;
#pragma unroll 4
                    for (int lb = 0; lb < lim; ++lb) {
                        const int b = 64 * rb + lb;
                        const int qb = __builtin_amdgcn_readlane(oq[rb], lb);
                        const double mb = rdlane(mj[rb], lb);
#pragma unroll
                        for (int r = 0; r < R; ++r) {
                            const int a = lane + 64 * r;
                            if (a < nf && a >= b && a != pj && b != pj) {
                                const int e = tri(oq[r], qb);
                                M[e] = M[e] - ma[r] * mb;
                            }
                        }
                    }
                }
                lds_sync();
                if (lane == 0) sh.ord[pj] = sh.ord[nf - 1];  // the last position fills the gap
                lds_sync();
                --nf;
            }
        }
    }
    lds_sync();
    return capped;
}


// ---- the QP of books of more than 32 names, on the whole workgroup ------------------------------
// The method, start point and pivot rules of qp_setup + qp_wave, laid out for 256 threads: thread
// t owns member row a = t & 127 and column half h = t >> 7 (columns 64h .. 64h + 63) of
// M = S_FF^-1 in REGISTERS, M embedded in the full 128 x 128 index space with the rows and columns
// of bound members and non-members exactly zero; S stays packed in LDS.  The bound set (and which
// bound) is tracked as uniform bit masks, so S_FB w_B, the bound weight sum and the multipliers
// need no gather.  Every product with M is a register mat-vec against a vector broadcast from
// LDS (the two halves' partials summed through LDS), and the active-set changes move no data:
//   join j (bordering):  u = M s (s = S[.][j]), d = S_jj - s'u, M <- M + u~ u~' / d with
//                        u~ = u - e_j (u_j = 0: row j of M is zero);
//   leave j (deflation): M <- M - m m' / m_jj (m = M[.][j]), then row and column j set to 0.
// Every update is one FMA per element with the row factor (x_a r) precomputed; M is symmetric to
// rounding, so a published ROW serves as the column (the optimum is unique: only the end point is
// compared, rel 1e-9).  The sweep operator builds M = S^-1 in the same layout, one published row
// per pivot.  Returns true if the iteration cap was hit (or S is not finite: weights NaN).
__device__ __forceinline__ void blk_sum3(double (&red)[4][4], double& x, double& y, double& z) {
    x = wave_sum(x);
    y = wave_sum(y);
    z = wave_sum(z);
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[wv][0] = x;
        red[wv][1] = y;
        red[wv][2] = z;
    }
    __syncthreads();
    x = ((red[0][0] + red[1][0]) + red[2][0]) + red[3][0];
    y = ((red[0][1] + red[1][1]) + red[2][1]) + red[3][1];
    z = ((red[0][2] + red[1][2]) + red[2][2]) + red[3][2];
}

// lexicographic (v, code) minimum over the workgroup, in every thread
__device__ __forceinline__ void blk_argmin(QpLds& q, double& v, int& code) {
    wave_argmin(v, code);
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        q.red[5][wv][0] = v;
        q.code[wv] = code;
    }
    __syncthreads();
    v = q.red[5][0][0];
    code = q.code[0];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
        const double v2 = q.red[5][w][0];
        const int c2 = q.code[w];
        if (v2 < v || (v2 == v && c2 < code)) { v = v2; code = c2; }
    }
}

__device__ __forceinline__ bool mbit(const u64 (&m)[2], int b) {
    return (m[b >> 6] >> (b & 63)) & 1ull;
}

template <int KM>
__device__ __noinline__ bool qp_block(Shared<KM>& sh, const int n, const double lo,
                                     const double hi, int64_t* stamps) {
    static_assert(KM == 128 && kT == 256, "qp_block: 128 member rows x 2 column halves");
    QpLds& q = sh.u.qp;
    // the column half is uniform per wave: column indices, their LDS addresses and the S row
    // reads of the bordering step are scalar
    const int tid = threadIdx.x, a = tid & 127;
    const int h = __builtin_amdgcn_readfirstlane(tid >> 7), b0 = 64 * h;
    const int wv = tid >> 6, lane = tid & 63;
    const bool mem = a < n;
    double Mr[64];
    int bad = 0;
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        const int b = b0 + i;
        Mr[i] = mem && b < n ? sh.S[tri(a, b)] : 0.0;
        bad |= !__builtin_isfinite(Mr[i]);
    }
    if (__syncthreads_or(bad)) {
        if (h == 0 && mem) sh.w[a] = __builtin_nan("");
        __syncthreads();
        return true;
    }
    // Block sweep, four pivots K = [k, k + 4) per published block (sweeps compose):
    //   A_KK <- -B^-1,  A_aK <- A_aK B^-1,  A_Kb <- B^-1 A_Kb,  A_ab <- A_ab - A_aK B^-1 A_Kb
    // with B = A_KK (identity past n).  After all blocks A = -S^-1.  Each thread sweeps B in
    // registers; row a then needs four coefficients: c = A_aK B^-1 off the block, and on it
    // (a = k + p) c = e_p - B^-1[p] so the same four FMAs per element give B^-1 A_Kb.
    for (int k = 0; k < n; k += 4) {
        double (*pub)[128] = q.pubk[(k >> 2) & 1];
        if (a >= k && a < k + 4) {
#pragma unroll
            for (int i = 0; i < 64; ++i) pub[a - k][b0 + i] = Mr[i];
        }
        __syncthreads();
        double B[4][4];
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y)
                B[x][y] = k + x < n && k + y < n ? pub[x][k + y] : (x == y ? 1.0 : 0.0);
#pragma unroll
        for (int p = 0; p < 4; ++p) {                  // B <- -B^-1
            const double r = 1.0 / B[p][p];
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int y = 0; y < 4; ++y)
                    if (x != p && y != p) B[x][y] = __builtin_fma(-B[x][p] * r, B[p][y], B[x][y]);
#pragma unroll
            for (int x = 0; x < 4; ++x)
                if (x != p) { B[x][p] *= r; B[p][x] *= r; }
            B[p][p] = -r;
        }
        const bool ink = a >= k && a < k + 4;
        double cg[4], cv[4];                           // update coefficients, block-column values
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            double c = 0.0;                            // A_aK B^-1 = -(A_aK (-B^-1))
#pragma unroll
            for (int x = 0; x < 4; ++x) c = __builtin_fma(-pub[x][a], B[x][y], c);
            double bp = 0.0;                           // -B^-1[a - k][y]
#pragma unroll
            for (int x = 0; x < 4; ++x) bp = a - k == x ? B[x][y] : bp;
            cv[y] = ink ? bp : c;
            cg[y] = ink ? bp + (a - k == y ? 1.0 : 0.0) : c;
        }
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            double pb[4][4];
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int y = 0; y < 4; ++y) pb[x][y] = pub[x][b0 + 4 * g + y];
            if (b0 + 4 * g == k) {
#pragma unroll
                for (int y = 0; y < 4; ++y) Mr[4 * g + y] = cv[y];
            } else {
#pragma unroll
                for (int y = 0; y < 4; ++y) {
                    double v = Mr[4 * g + y];
#pragma unroll
                    for (int x = 0; x < 4; ++x) v = __builtin_fma(-cg[x], pb[x][y], v);
                    Mr[4 * g + y] = v;
                }
            }
        }
    }
    const double fin = mem ? -1.0 : 0.0;               // M = S^-1; rows past n exactly 0
#pragma unroll
    for (int i = 0; i < 64; ++i) Mr[i] *= fin;
    if (stamps && tid == 0) stamps[6] = wall_clock64();

    u64 bnd[2] = {0ull, 0ull}, bhi[2] = {0ull, 0ull};   // uniform: bound members, those at hi
    double wa = mem ? 1.0 / n : 0.0;                    // own member's weight
    int nf = n;
    bool capped = false;
    const int max_it = 4 * n + 8;
    int it = 0;
    for (; it < max_it; ++it) {
        if (nf == 0) break;
        if (it == max_it - 1) capped = true;
        const bool ba = mem && mbit(bnd, a), fa = mem && !ba;
        // c = S_FB w_B and the bound weight sum, bound members in ascending order
        double ca = 0.0, bs = 0.0;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            u64 m = bnd[r];
            while (m) {
                const int b = 64 * r + __builtin_ctzll(m);
                m &= m - 1ull;
                const double wb = mbit(bhi, b) ? hi : lo;
                bs += wb;
                if (h == 0) ca = ca + sh.S[tri(a, b)] * wb;
            }
        }
        if (h == 0) q.vc[a] = fa ? ca : 0.0;
        __syncthreads();
        double p1 = 0.0, p2 = 0.0;                     // y1 = M 1_F, y2 = M c
#pragma unroll
        for (int i = 0; i < 64; ++i) {
            p1 = p1 + Mr[i];
            p2 = __builtin_fma(Mr[i], q.vc[b0 + i], p2);
        }
        q.part[1][h][a] = p1;
        q.part[2][h][a] = p2;
        __syncthreads();
        const double y1 = q.part[1][0][a] + q.part[1][1][a];
        const double y2 = q.part[2][0][a] + q.part[2][1][a];
        double s1 = h == 0 && fa ? y1 : 0.0, s2 = h == 0 && fa ? y2 : 0.0, z0 = 0.0;
        blk_sum3(q.red[0], s1, s2, z0);
        const double lam = -((1.0 - bs) + s2) / s1;
        const double xa = -y2 - lam * y1;
        const bool infeas = __syncthreads_or(fa && (!(xa >= lo) || !(xa <= hi)));
        if (!infeas) {
            // feasible: take x; release the bound member with the most negative multiplier
            // g_j = S[j][.] w + lam, one bound member per wave at a time
            if (fa) wa = xa;
            if (h == 0) q.vw[a] = wa;
            __syncthreads();
            double vmin = __builtin_inf();
            int jmin = 0x7fffffff, ib = 0;
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                u64 m = bnd[r];
                while (m) {
                    const int j = 64 * r + __builtin_ctzll(m);
                    m &= m - 1ull;
                    if ((ib++ & 3) != wv) continue;
                    double g = 0.0;
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const int b = lane + 64 * e;
                        if (b < n) g = g + sh.S[tri(j, b)] * q.vw[b];
                    }
                    g = wave_sum(g) + lam;
                    const double v = mbit(bhi, j) ? -g : g;
                    if (v < vmin) { vmin = v; jmin = j; }
                }
            }
            blk_argmin(q, vmin, jmin);
            if (!(vmin < 0.0)) break;
            // bordering by member j: s = S[.][j], u = M s, d = S_jj - s'u
            const int j = __builtin_amdgcn_readfirstlane(jmin);
            double up = 0.0;
#pragma unroll
            for (int i = 0; i < 64; ++i) {
                const int b = b0 + i;
                up = __builtin_fma(Mr[i], b < n ? sh.S[tri(j, b)] : 0.0, up);
            }
            q.part[3][h][a] = up;
            __syncthreads();
            const double ua = q.part[3][0][a] + q.part[3][1][a];    // 0 off the free set
            double su = h == 0 && fa ? sh.S[tri(a, j)] * ua : 0.0, z1 = 0.0, z2 = 0.0;
            blk_sum3(q.red[1], su, z1, z2);
            const double rd = 1.0 / (sh.S[tri(j, j)] - su);
            const double ut = a == j ? -1.0 : ua;
            if (h == 0) q.vu[a] = ut;
            __syncthreads();
            const double utr = ut * rd;
#pragma unroll
            for (int i = 0; i < 64; ++i) Mr[i] = __builtin_fma(utr, q.vu[b0 + i], Mr[i]);
            bnd[j >> 6] &= ~(1ull << (j & 63));
            bhi[j >> 6] &= ~(1ull << (j & 63));
            ++nf;
        } else {
            // ratio test: the first member (ascending index) to hit its bound along x - w
            double amin = __builtin_inf();
            int code = 0x7fffffff;                     // 2 * member + (bound is hi)
            if (h == 0 && fa) {
                const double pq = xa - wa;
                if (xa < lo && pq < 0) {
                    const double al = (lo - wa) / pq;
                    if (al < 1.0) { amin = al; code = 2 * a; }
                } else if (xa > hi && pq > 0) {
                    const double al = (hi - wa) / pq;
                    if (al < 1.0) { amin = al; code = 2 * a + 1; }
                }
            }
            blk_argmin(q, amin, code);
            const bool hit = code != 0x7fffffff;
            const double alpha = hit ? amin : 1.0;
            if (fa) wa = wa + alpha * (xa - wa);
            if (hit) {
                // deflation of member jb: m = M[.][jb] (= row jb)
                const int jb = __builtin_amdgcn_readfirstlane(code >> 1);
                const bool tohi = code & 1;
                if (a == jb) wa = tohi ? hi : lo;
                bnd[jb >> 6] |= 1ull << (jb & 63);
                if (tohi) bhi[jb >> 6] |= 1ull << (jb & 63);
                double* pub = q.pubk[0][0];
                if (a == jb) {
#pragma unroll
                    for (int i = 0; i < 64; ++i) pub[b0 + i] = Mr[i];
                }
                __syncthreads();
                const double mr = pub[a] * (1.0 / pub[jb]);
#pragma unroll
                for (int i0 = 0; i0 < 64; i0 += 16) {
                    double pb[16];
#pragma unroll
                    for (int i = 0; i < 16; ++i) pb[i] = pub[b0 + i0 + i];
                    if (jb >= b0 + i0 && jb < b0 + i0 + 16) {
#pragma unroll
                        for (int i = 0; i < 16; ++i)
                            Mr[i0 + i] = b0 + i0 + i == jb ? 0.0
                                                            : __builtin_fma(-pb[i], mr, Mr[i0 + i]);
                    } else {
#pragma unroll
                        for (int i = 0; i < 16; ++i)
                            Mr[i0 + i] = __builtin_fma(-pb[i], mr, Mr[i0 + i]);
                    }
                }
                if (a == jb) {
#pragma unroll
                    for (int i = 0; i < 64; ++i) Mr[i] = 0.0;
                }
                --nf;
            }
        }
    }
    if (h == 0 && mem) sh.w[a] = wa;
    if (stamps && tid == 0) stamps[7] = it;
    __syncthreads();
    return capped;
}

// determine_weights for one book: [rows][ld] returns (k columns, NaN = missing) -> covariance
// (an output) and weights
__global__ __launch_bounds__(kT) void weights_kernel(const double* R, int64_t rows, int64_t ld,
                                                     int k, double lo, double hi, double* w,
                                                     double* cov, int32_t* status) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    Shared<kMaxK>& sh = *reinterpret_cast<Shared<kMaxK>*>(smem_raw);
    auto get = [&](int m, int64_t row) -> double {
        return row < rows ? R[row * ld + m] : __builtin_nan("");
    };
    if (k > 32) book_cov_mfma(sh, k, rows, get);
    else book_cov(sh, k, rows, get);
    const int tid = threadIdx.x;
    for (int e = tid; e < k * k; e += kT) cov[e] = sh.S[tri(e / k, e % k)];
    bool capped = false;
    if (k * hi <= 1.0) {
        if (tid < k) sh.w[tid] = hi;
    } else if (k * lo >= 1.0) {
        if (tid < k) sh.w[tid] = lo;
    } else if (k <= 32) {            // the solve rebalance_kernel<32> runs (headline books)
        const bool ok = qp_setup(sh, k);
        if (!ok) capped = true;
        else if (tid < 64) capped = qp_wave(sh, k, lo, hi);
    } else {
        capped = qp_block(sh, k, lo, hi, nullptr);
    }
    __syncthreads();
    if (tid < k) w[tid] = sh.w[tid];
    if (tid == 0) status[0] = capped ? 1 : 0;
}

// One workgroup per (rebalance date i = blockIdx.x, book side = blockIdx.y): side 0 the long
// book (k largest predictions), side 1 the short book (k smallest).
template <int KM>
__global__ __launch_bounds__(kT) void rebalance_kernel(RebArgs r) {
    AFM_TAIL_PRIO_SET();
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    Shared<KM>& sh = *reinterpret_cast<Shared<KM>*>(smem_raw);
    const int tid = threadIdx.x;
    const int64_t i = blockIdx.x;
    const int side = blockIdx.y;
    const int64_t t = r.dates[i];
    const int64_t tp = i > 0 ? r.dates[i - 1] : -1;
    const int64_t tn = i + 1 < r.nd ? r.dates[i + 1] : -1;
    const int nw = (int)((r.A + 63) / 64);

    // ---- prediction presence rows (prev, cur, next) by ballot; candidate keys of date t in
    // registers (asset j * kT + tid) when the panel is narrow enough ---------------------------
    constexpr int KR = 48;                           // register keys: A <= 12288
    const bool regk = r.A <= (int64_t)KR * kT;
    u64 ks[KR];
#pragma unroll
    for (int j = 0; j < KR; ++j) ks[j] = 0ull;
    int nc = 0;
    {
        for (int64_t a0 = 0; a0 < (int64_t)nw * 64; a0 += kT) {
            const int64_t a = a0 + tid;
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const int64_t tq = q == 0 ? tp : (q == 1 ? t : tn);
                bool has = false;
                if (tq >= 0 && a < r.A) {
                    const double v = r.pred[tq * r.lda + a];
                    has = v == v;
                }
                const u64 m = __ballot(has);
                if ((tid & 63) == 0) sh.pw[q][a >> 6] = m;
            }
        }
    }
    if (regk) {
#pragma unroll
        for (int j = 0; j < KR; ++j) {
            const int64_t a = (int64_t)j * kT + tid;
            if (a < r.A) {
                const double v = r.pred[t * r.lda + a];
                if (v == v && bit_at(r.trad, r.lda, t, a)) {
                    ks[j] = okey(v);
                    ++nc;
                }
            }
        }
    } else {
        for (int64_t a = tid; a < r.A; a += kT) {
            double v = r.pred[t * r.lda + a];
            nc += (v == v && bit_at(r.trad, r.lda, t, a)) ? 1 : 0;
        }
    }
    int ex;
    const int ncand = block_scan(nc, sh.scan, &ex);
    const int k = ncand < 2 * r.top_n ? ncand / 2 : r.top_n;
    if (k > KM) {
        if (tid == 0) { r.status[i] = 2; if (side == 0) r.k_out[i] = k; }
        return;
    }
    if (tid == 0 && side == 0) r.k_out[i] = k;

    if (r.stamps && tid == 0) r.stamps[(i * 2 + side) * 8 + 0] = wall_clock64();
    const bool largest = side == 0;
    if (k > 0 && regk) {
        if (!select_top_reg<KR>(sh, ks, k, largest, sh.book))
            select_top(r, sh, t, k, largest, sh.book);
    } else if (k > 0) {
        select_top(r, sh, t, k, largest, sh.book);
    }
    __syncthreads();

    const int64_t hlo = r.window > 0 ? (t - r.window > 0 ? t - r.window : 0) : r.h_t0;
    const int64_t hhi = r.window > 0 ? t : r.h_t1;
    if (r.stamps && tid == 0) r.stamps[(i * 2 + side) * 8 + 1] = wall_clock64();
    const int* bk = sh.book;
    // ---- pairwise-complete covariance of the book's history window ------------------------
    const int64_t rows = hhi - hlo;
    auto gather = [&](int m, int64_t row) -> double {
        const int64_t th = hlo + row;
        const int64_t tt = th < hhi ? th : hlo;              // loads always in bounds
        const int a = bk[m];
        const u64 wb = r.hbits[(tt >> 6) * r.lda + a];
        const double hv = r.hist[tt * r.lda + a];
        return (th < hhi && ((wb >> (tt & 63)) & 1ull)) ? hv : __builtin_nan("");
    };
    if (r.probe & 2) {
        for (int e = tid; e < k * (k + 1) / 2; e += kT) {
            int a = 0, q = e;
            while (q > a) { q -= a + 1; ++a; }
            sh.S[e] = a == q ? 1e-4 : 1e-6;
        }
        __syncthreads();
    } else if (r.histT != nullptr) {
        if constexpr (KM == kMaxK) {
            // each member's window is contiguous in the member-major panel: coalesced staging
            if (r.stamps && tid == 0) r.stamps[(i * 2 + side) * 8 + 5] = wall_clock64();
            // captured by value: the covariance is a called function, and references into the
            // kernel arguments would be reloaded at every element
            const double* hT = r.histT + (hlo - r.hT0);
            const int64_t ld = r.hTn;
            auto fromT = [hT, ld, bk, rows](int m, int64_t row) -> double {
                const double x = hT[(int64_t)bk[m] * ld + (row < rows ? row : 0)];
                return row < rows ? x : __builtin_nan("");
            };
            if (k > 32) book_cov_mfma(sh, k, rows, fromT);
            else book_cov(sh, k, rows, fromT);
        }
    } else if (k * (k + 1) / 2 <= kT || r.hscr == nullptr) {
        if constexpr (KM == kMaxK) {
            if (k > 32) book_cov_mfma(sh, k, rows, gather);
            else book_cov(sh, k, rows, gather);             // one pass over the member pairs
        } else {
            book_cov(sh, k, rows, gather);
        }
    } else {
        // several passes: gather the members' window once into a contiguous [member][row]
        // scratch block, which every pass then stages with coalesced reads
        double* H = r.hscr + (i * 2 + side) * (int64_t)r.top_n * r.hrows;
        // (16 uncoalesced loads in flight per thread: the rows of one member are lda apart)
        const int ne = k * (int)rows, nr = (int)rows;
        constexpr int G = 16;
        for (int e0 = 0; e0 < ne; e0 += G * kT) {
            double v[G];
#pragma unroll
            for (int j = 0; j < G; ++j) {
                const int e = e0 + j * kT + tid;
                const int m = (unsigned)e / (unsigned)nr;
                v[j] = e < ne ? gather(m, e - m * nr) : 0.0;
            }
#pragma unroll
            for (int j = 0; j < G; ++j) {
                const int e = e0 + j * kT + tid;
                if (e < ne) H[e] = v[j];
            }
        }
        __syncthreads();
        if (r.stamps && tid == 0) r.stamps[(i * 2 + side) * 8 + 5] = wall_clock64();
        auto fromH = [&](int m, int64_t row) -> double {
            return row < rows ? H[m * rows + row] : __builtin_nan("");
        };
        if constexpr (KM == kMaxK) {
            if (k > 32) book_cov_mfma(sh, k, rows, fromH);  // masked SYRKs on fp64 MFMA
            else book_cov(sh, k, rows, fromH);
        } else {
            book_cov(sh, k, rows, fromH);
        }
    }

    // ---- exact box-constrained QP (primal active set, wave 0) -----------------------------
    if (r.stamps && tid == 0) r.stamps[(i * 2 + side) * 8 + 2] = wall_clock64();
    bool capped = false;
    if (k > 0 && k * r.hi <= 1.0) {
        if (tid < k) sh.w[tid] = r.hi;
    } else if (k > 0 && k * r.lo >= 1.0) {
        if (tid < k) sh.w[tid] = r.lo;
    } else if (k > 0 && (r.probe & 1)) {
        if (tid < k) sh.w[tid] = 1.0 / k;
    } else if (k > 0) {
        if constexpr (KM == kMaxK) {
            capped = qp_block(sh, k, r.lo, r.hi,
                              r.stamps ? r.stamps + (i * 2 + side) * 8 : nullptr);
        } else {
            const bool ok = qp_setup(sh, k);
            if (r.stamps && tid == 0) r.stamps[(i * 2 + side) * 8 + 6] = wall_clock64();
            if (!ok) capped = true;
            else if (tid < 64) capped = qp_wave(sh, k, r.lo, r.hi);
        }
    }
    if (capped && tid == 0) atomicOr(&r.status[i], 1);
    __syncthreads();
    // ---- outputs for this book -----------------------------------------------------------
    if (r.stamps && tid == 0) r.stamps[(i * 2 + side) * 8 + 3] = wall_clock64();
    double* wout = r.weights + (i * 2 + side) * kMaxK;
    int32_t* bout = r.books + (i * 2 + side) * kMaxK;
    if (tid < k) {
        wout[tid] = sh.w[tid];
        bout[tid] = bk[tid];
        const double tw = r.tmr[t * r.lda + bk[tid]] * sh.w[tid];   // tmr * w (book order)
        sh.x[tid] = tw == tw ? tw : 0.0;                            // nansum
        sh.c[tid] = sh.w[tid] * r.close[t * r.lda + bk[tid]];       // w * price
    }
    __syncthreads();
    if (tid == 0) {
        r.sums[i * 4 + side] = pairwise_dense(sh.x, k);
        double den = 0.0;                                           // builtin sum(): 0 + ...
        for (int a = 0; a < k; ++a) den = den + sh.c[a];
        r.sums[i * 4 + 2 + side] = den;
    }
    // union positions of the members vs the previous / next rebalance date
    if (tid < k) {
        const int a = bk[tid];
        const int wa = a >> 6, ba = a & 63;
        for (int q = 0; q < 2; ++q) {
            const int other = q == 0 ? 0 : 2;                       // prev row / next row
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
    if (r.stamps && tid == 0) r.stamps[(i * 2 + side) * 8 + 4] = wall_clock64();
    if (side == 0 && tid < 2) {
        const int other = tid == 0 ? 0 : 2;
        int64_t tot = 0;
        for (int wi = 0; wi < nw; ++wi) tot += __popcll(sh.pw[other][wi] | sh.pw[1][wi]);
        r.usize[i * 2 + tid] = tot;
    }
}

// ---- sequential value / turnover recursion (KKT:864-892) ----------------------------------
// The turnover is numpy's pairwise sum over the union-aligned vector |cur - new| (KKT:839), which
// is zero except at the books' members.  Zero slots contribute exact +0.0 (every term is
// |.| >= 0), so the summation tree restricted to the members is a DAG of binary adds over the
// member terms whose shape depends only on the union length and the members' positions -- not
// on the portfolio value.  turnover_terms_kernel (parallel over dates) compiles each date's DAG
// into a record of LEVELS (every add of level l depends only on lower levels); the sequential
// scan then evaluates one date as: term values (lane-parallel), one lane-parallel step per DAG
// level, the value update -- all out of LDS, with records staged a chunk of dates ahead.
constexpr int kMaxTerms = 4 * kMaxK;        // terms of one date (<= 2 books x 2 dates x k)
// DAG depth <= 16 (one accumulator of a 128-wide leaf) + 3 + 7 (tail) + log2(65536 / 128) = 35
constexpr int kMaxLevels = 64;
constexpr int kRec = 4 + 2 * kMaxTerms + kMaxLevels;   // record words (fixed global stride)
// record: [0] m (terms; -1: no turnover that date) [1] nint (adds) [2] L (levels) [3] unused,
//         [4, 4+m) term codes (3 * prev side + new side; side 2 = absent),
//         [4+m, 4+m+nint) adds in level order: left | right << 16 (node ids: terms 0..m-1,
//         add q -> m + q), then L cumulative add counts per level.
// The full summation tree of numpy's pairwise_sum over n slots (numpy/_core/src/umath/
// loops_utils.h.src): a node of more than 128 slots adds its halves (n2 = n / 2 rounded down to a
// multiple of 8); a block of 8 <= n <= 128 slots runs 8 strided accumulators (chains, a[j] then
// += a[j + 8c]), combines them ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) and adds the
// n % 8 tail slots one by one; a block of n < 8 slots adds them one by one onto 0.  Restricted to
// the member terms, the DAG's adds are exactly the lowest common ancestors of the terms that are
// consecutive in the tree's in-order, so it is the Cartesian tree of those ancestors' depths --
// built here lane-parallel (round 4; a one-lane recursive build took ~200 us per date).
// Buffered reduction over more than 8192 slots: np_key / np_lca_depth below.
struct PwBlock {
    int64_t lo, len;
    int depth;
};
__device__ __forceinline__ PwBlock pw_block(int64_t n, int64_t pos) {
    int64_t lo = 0, len = n;
    int d = 0;
    while (len > 128) {
        int64_t n2 = len / 2;
        n2 -= n2 % 8;
        if (pos < lo + n2) len = n2;
        else { lo += n2; len -= n2; }
        ++d;
    }
    return {lo, len, d};
}
// the in-order key of a slot inside its block: accumulator-major in the body, then the tail
__device__ __forceinline__ int pw_inkey(const PwBlock& b, int64_t pos) {
    const int off = (int)(pos - b.lo);
    if (b.len < 8) return off;
    const int body = (int)(b.len - b.len % 8);
    return off < body ? (off % 8) * 16 + off / 8 : 128 + (off - body);
}
// depth (root 0) of the lowest common ancestor of the slots p and q, p before q in in-order
__device__ int pw_lca_depth(int64_t n, int64_t p, int64_t q);
// np.add.reduce over n slots (what Series.sum runs): the identity 0.0, then the pairwise sums of
// consecutive 8192-slot buffers (NPY_BUFSIZE) added one by one -- over 8192 slots the sum is NOT
// one pairwise tree (config C's id unions are ~9,000-10,000 long; oracle np_sum, checked against
// numpy itself in tests/test_oracle_golden.py).  The full tree: a left-deep chain over the
// buffers (buffer c joins at depth K - 1 - c), buffer c's pairwise tree rooted at depth K - c
// (buffer 0: K, below the add of the identity).
constexpr int64_t kNpBuf = 8192;
__device__ __forceinline__ int np_key(int64_t n, int64_t pos) {
    const int64_t c0 = pos - pos % kNpBuf;
    const int64_t cl = n - c0 < kNpBuf ? n - c0 : kNpBuf;
    const PwBlock b = pw_block(cl, pos - c0);
    return (int)((c0 + b.lo) << 8) | pw_inkey(b, pos - c0);
}
__device__ int np_lca_depth(int64_t n, int64_t p, int64_t q) {
    const int K = (int)((n + kNpBuf - 1) / kNpBuf);
    const int cp = (int)(p / kNpBuf), cq = (int)(q / kNpBuf);
    if (cp != cq) return K - 1 - cq;
    const int64_t c0 = (int64_t)cq * kNpBuf;
    const int64_t cl = n - c0 < kNpBuf ? n - c0 : kNpBuf;
    return (cq == 0 ? K : K - cq) + pw_lca_depth(cl, p - c0, q - c0);
}
__device__ int pw_lca_depth(int64_t n, int64_t p, int64_t q) {
    int64_t lo = 0, len = n;
    int d = 0;
    while (len > 128) {
        int64_t n2 = len / 2;
        n2 -= n2 % 8;
        const bool lp = p < lo + n2, lq = q < lo + n2;
        if (lp != lq) return d;
        if (lp) len = n2;
        else { lo += n2; len -= n2; }
        ++d;
    }
    const int op = (int)(p - lo), oq = (int)(q - lo), nb = (int)len;
    if (nb < 8) return d + (nb - 1 - oq);               // the add of slot q onto the running sum
    const int nt = nb % 8, body = nb - nt;
    if (oq >= body) return d + (nt - 1 - (oq - body));  // q's tail add
    const int jp = op % 8, jq = oq % 8;
    if (jp == jq) return d + nt + 3 + (body / 8 - 1 - oq / 8);   // q's add in its chain
    if (jp / 2 == jq / 2) return d + nt + 2;
    if (jp / 4 == jq / 4) return d + nt + 1;
    return d + nt;
}

// Steps i are grouped in sequences of `seq` (one bootstrap path each; seq = nd for the plain
// rebalance sequence); the book of step i is book slot ix(i) (idx = nullptr: slot i).  upos /
// usize are per step.
// Two kernels build the records (round 5): turnover_terms_wave_kernel, one wave per step with
// every stage in registers, for steps whose books (this step's and the previous one's) hold at
// most kWaveK names -- the headline's top_n = 10 and every bootstrap path step of config E -- and
// turnover_terms_kernel below, a persistent grid over the remaining steps (larger books: LDS
// arrays of kMaxTerms).  The records differ only in the order of the adds inside a DAG level
// (any order within a level evaluates the same additions), so the turnover is bitwise the same.
constexpr int kWaveK = 16;                   // 2 books x 2 dates x 16 <= 64 terms: one per lane
__global__ __launch_bounds__(64) void turnover_terms_kernel(int64_t nd, const int32_t* k_out,
                                                            const int32_t* books,
                                                            const int32_t* upos,
                                                            const int64_t* usize, int32_t* rec,
                                                            int32_t* rlen, const int32_t* idx,
                                                            int64_t seq, const int32_t* rest) {
    AFM_SCAN_PRIO_SET();
    __shared__ int pos_s[kMaxTerms], code_s[kMaxTerms], pos_o[kMaxTerms], code_o[kMaxTerms];
    __shared__ int key_s[kMaxTerms], dep[kMaxTerms], lch[kMaxTerms], rch[kMaxTerms];
    __shared__ int hgt[kMaxTerms], newid[kMaxTerms], lcount[kMaxLevels + 1];
    __shared__ int cnt, nlev;
    const int nrest = rest[0];                       // the steps turnover_terms_wave_kernel left
    for (int j = blockIdx.x; j < nrest; j += gridDim.x) {       // (uniform per workgroup)
    const int64_t i = rest[1 + j];
    const int tid = threadIdx.x;
    int32_t* R = rec + i * kRec;
    __syncthreads();                                 // the previous step's LDS reads are done
    if (tid == 0) cnt = 0;
    __syncthreads();
    const int64_t si = idx ? idx[i] : i;             // book slots of this and the previous step
    const int64_t sp = i % seq == 0 ? -1 : (idx ? idx[i - 1] : i - 1);
    const bool active = sp >= 0 && k_out[sp] > 0;    // current_positions.dropna().empty -> 0
    // both dates' books into LDS first (round 4: the membership tests below read them ~4k times
    // per lane; from global memory each was a dependent load, ~0.2 ms per workgroup)
    __shared__ int bk_cur[2 * kMaxK], bk_prev[2 * kMaxK];
    int k = 0, kp = 0;
    if (active) {
        k = k_out[si];
        kp = k_out[sp];
        for (int e = tid; e < 2 * k; e += 64) bk_cur[e] = books[(si * 2 + e / k) * kMaxK + e % k];
        for (int e = tid; e < 2 * kp; e += 64) bk_prev[e] = books[(sp * 2 + e / kp) * kMaxK + e % kp];
    }
    __syncthreads();
    if (active) {
        for (int e = tid; e < 2 * kp; e += 64) {     // previous members predicted today
            const int side = e / kp, q = e % kp;
            const int a = bk_prev[e];
            const int pz = upos[(((i - 1) * 2 + side) * 2 + 1) * kMaxK + q];
            if (pz < 0) continue;
            int ns = 2;
            for (int q2 = 0; q2 < 2 * k; ++q2)
                if (bk_cur[q2] == a) ns = q2 / k;
            const int slot = atomicAdd(&cnt, 1);
            pos_s[slot] = pz;
            code_s[slot] = side * 3 + ns;
        }
        for (int e = tid; e < 2 * k; e += 64) {      // today's members predicted yesterday only
            const int side = e / k, q = e % k;
            const int a = bk_cur[e];
            const int pz = upos[((i * 2 + side) * 2 + 0) * kMaxK + q];
            if (pz < 0) continue;
            bool inprev = false;
            for (int q2 = 0; q2 < 2 * kp; ++q2)
                if (bk_prev[q2] == a) inprev = true;
            if (inprev) continue;
            const int slot = atomicAdd(&cnt, 1);
            pos_s[slot] = pz;
            code_s[slot] = 2 * 3 + side;
        }
    }
    __syncthreads();
    const int m = cnt;
    const int64_t n = usize[i * 2 + 0];
    for (int e = tid; e < m; e += 64) key_s[e] = np_key(n, pos_s[e]);   // the tree's in-order
    __syncthreads();
    for (int e = tid; e < m; e += 64) {
        int r = 0;
        for (int f = 0; f < m; ++f) r += key_s[f] < key_s[e];
        pos_o[r] = pos_s[e];
        code_o[r] = code_s[e];
    }
    __syncthreads();
    // internal node k (0 <= k < m - 1) = the LCA of in-order terms k and k + 1
    const int ni = m > 1 ? m - 1 : 0;
    for (int k = tid; k < ni; k += 64) dep[k] = np_lca_depth(n, pos_o[k], pos_o[k + 1]);
    __syncthreads();
    // Cartesian tree: the left child of k is the shallowest node between the nearest shallower
    // node on its left and k (or term k), the right child likewise (or term k + 1); child ids:
    // term t -> t, node k -> m + k
    for (int k = tid; k < ni; k += 64) {
        const int dk = dep[k];
        int best = -1, bd = 1 << 30;
        for (int l = k - 1; l >= 0 && dep[l] > dk; --l)
            if (dep[l] < bd) { bd = dep[l]; best = l; }
        lch[k] = best < 0 ? k : m + best;
        best = -1;
        bd = 1 << 30;
        for (int r = k + 1; r < ni && dep[r] > dk; ++r)
            if (dep[r] < bd) { bd = dep[r]; best = r; }
        rch[k] = best < 0 ? k + 1 : m + best;
        hgt[k] = 1;
    }
    __syncthreads();
    // heights (the DAG level of an add: 1 + its children's), relaxed until they settle: a height
    // is at most ni, so ni + 1 rounds always settle (the loop exits at the first quiet round)
    if (tid == 0) nlev = 0;
    for (int it = 0; it < ni + 1; ++it) {
        bool ch = false;
        for (int k = tid; k < ni; k += 64) {
            const int a = lch[k], b = rch[k];
            const int ha = a < m ? 0 : hgt[a - m], hb = b < m ? 0 : hgt[b - m];
            const int h = (ha > hb ? ha : hb) + 1;
            if (h != hgt[k]) { hgt[k] = h; ch = true; }
        }
        __syncthreads();
        if (__syncthreads_or(ch) == 0) break;
    }
    for (int k = tid; k < ni; k += 64) atomicMax(&nlev, hgt[k]);
    __syncthreads();
    if (nlev > kMaxLevels) {
        // a DAG deeper than the record's level table (kMaxLevels): an error record (m = -2) the
        // scan turns into a NaN turnover -- and so a NaN value path from this step on -- instead
        // of writing the level counts out of bounds
        if (tid == 0) {
            R[0] = -2;
            R[1] = 0;
            R[2] = 0;
            R[3] = 0;
            rlen[i] = 4;
        }
        continue;
    }
    for (int l = tid; l <= kMaxLevels; l += 64) lcount[l] = 0;
    __syncthreads();
    for (int k = tid; k < ni; k += 64) atomicAdd(&lcount[hgt[k]], 1);
    __syncthreads();
    const int L = nlev;
    if (tid == 0) {
        int acc = 0;                                  // lcount[l] -> first slot of level l
        for (int l = 1; l <= L; ++l) { const int c = lcount[l]; lcount[l] = acc; acc += c; }
        R[0] = active ? m : -1;
        R[1] = ni;
        R[2] = L;
        R[3] = 0;
        rlen[i] = 4 + (active ? m : 0) + ni + L;
    }
    __syncthreads();
    for (int k = tid; k < ni; k += 64) newid[k] = atomicAdd(&lcount[hgt[k]], 1);
    __syncthreads();
    for (int e = tid; e < m; e += 64) R[4 + e] = code_o[e];
    for (int k = tid; k < ni; k += 64) {
        const int a = lch[k], b = rch[k];
        const int na = a < m ? a : m + newid[a - m];
        const int nb = b < m ? b : m + newid[b - m];
        R[4 + m + newid[k]] = na | (nb << 16);
    }
    for (int l = tid; l < L; l += 64) R[4 + m + ni + l] = lcount[l + 1];   // cumulative ends
    }
}

// One wave per step (books of <= kWaveK names): lane e < 2 kp holds the previous step's member e,
// lane 32 + e this step's member e; a member's term is its |cur - new| slot in the union (KKT:839).
// Every stage runs lane-parallel in registers (no LDS, no barrier), with loops over set lanes or
// over depth / level values instead of over all 64 lanes:
//  - membership: one readlane loop over the members of both dates;
//  - in-order rank: a readlane loop over the valid terms, then ds_permute to the sorted lane;
//  - Cartesian tree: the depths are LCA depths of one real tree, so two nodes of equal depth have
//    a shallower node between them -- the nearest not-deeper node on each side is the nearest
//    strictly shallower one, found by ballots over the depth values in ascending order; a
//    node's parent is the deeper of the two, and the children are scattered to their parent's
//    lane with ds_permute (the same tree turnover_terms_kernel builds by interval scans);
//  - heights: relaxation as in turnover_terms_kernel; level order: one ballot per level.
__device__ __forceinline__ int wv_read(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ int wv_pull(int v, int src) {           // v of lane src (any lane)
    return __builtin_amdgcn_ds_bpermute(src << 2, v);
}
__device__ __forceinline__ int wv_push(int v, int dst) {           // v to lane dst (others: 0)
    return __builtin_amdgcn_ds_permute(dst << 2, v);
}
__device__ __forceinline__ int wv_min(int v) {
    for (int o = 32; o >= 1; o >>= 1) { const int x = __shfl_xor(v, o, 64); v = x < v ? x : v; }
    return v;
}
__device__ __forceinline__ int wv_max(int v) {
    for (int o = 32; o >= 1; o >>= 1) { const int x = __shfl_xor(v, o, 64); v = x > v ? x : v; }
    return v;
}
// rest[0] counts the steps left to turnover_terms_kernel (a book over kWaveK names), rest[1 + j]
// lists them.  n < 2^31 (the hosts check).
__global__ __launch_bounds__(256) void turnover_terms_wave_kernel(int64_t nd, const int32_t* k_out,
                                                                  const int32_t* books,
                                                                  const int32_t* upos,
                                                                  const int64_t* usize,
                                                                  int32_t* rec, int32_t* rlen,
                                                                  const int32_t* idx, int64_t seq,
                                                                  int32_t* rest) {
    AFM_SCAN_PRIO_SET();
    const int lane = threadIdx.x & 63;
    const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
    const uint64_t above = lane < 63 ? (~0ull << (lane + 1)) : 0ull;
    const uint32_t useq = (uint32_t)seq;
    const int nwv = (int)(gridDim.x * (blockDim.x >> 6));
    for (int i = (int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)); i < (int)nd; i += nwv) {
        const bool first = (uint32_t)i % useq == 0;
        const int si = idx ? idx[i] : i;
        const int sp = first ? -1 : (idx ? idx[i - 1] : i - 1);
        const int k = k_out[si], kp = sp >= 0 ? k_out[sp] : 0;
        if (k > kWaveK || kp > kWaveK) {                           // (uniform in the wave)
            if (lane == 0) rest[1 + atomicAdd(rest, 1)] = i;
            continue;
        }
        int32_t* R = rec + (int64_t)i * kRec;
        if (sp < 0 || kp <= 0) {                                   // current_positions.dropna().empty
            if (lane == 0) {
                R[0] = -1;
                R[1] = 0;
                R[2] = 0;
                R[3] = 0;
                rlen[i] = 4;
            }
            continue;
        }
        const int64_t n = usize[(int64_t)i * 2 + 0];
        // members: lane e < 2 kp the previous books', lane 32 + e < 32 + 2 k this step's
        const bool isp = lane < 2 * kp, isc = lane >= 32 && lane - 32 < 2 * k;
        int a = -1, side = 0, pz = -1;
        if (isp) {        // a previous member predicted today: |pos_old - pos_new| at its new slot
            side = lane >= kp;
            const int q = lane - side * kp;
            a = books[((int64_t)sp * 2 + side) * kMaxK + q];
            pz = upos[((((int64_t)i - 1) * 2 + side) * 2 + 1) * kMaxK + q];
        }
        if (isc) {        // a member predicted yesterday only (not in yesterday's books)
            side = lane - 32 >= k;
            const int q = lane - 32 - side * k;
            a = books[((int64_t)si * 2 + side) * kMaxK + q];
            pz = upos[(((int64_t)i * 2 + side) * 2 + 0) * kMaxK + q];
        }
        int ns = 2;
        bool inprev = false;
        for (uint64_t b = __ballot(isp || isc); b; b &= b - 1) {   // (uniform loop)
            const int j = __builtin_ctzll(b);
            const int aj = wv_read(a, j), sj = wv_read(side, j);
            if (aj == a) {
                if (j >= 32) ns = sj;
                else inprev = true;
            }
        }
        const int code = isp ? side * 3 + ns : 2 * 3 + side;
        const bool valid = (isp || (isc && !inprev)) && pz >= 0;
        const uint64_t vm = __ballot(valid);
        const int m = __popcll(vm);
        const int key = valid ? np_key(n, pz) : 0x7fffffff;
        // rank by key among the valid lanes (keys of distinct slots are distinct); the invalid
        // lanes take the ranks after them, in lane order
        int r = 0;
        for (uint64_t b = vm; b; b &= b - 1) r += wv_read(key, __builtin_ctzll(b)) < key ? 1 : 0;
        if (!valid) r = m + __popcll(~vm & below);
        const int pos_o = wv_push(pz, r);
        const int code_o = wv_push(code, r);
        // internal node kk (kk < m - 1) = the LCA of in-order terms kk and kk + 1
        const int ni = m > 1 ? m - 1 : 0;
        const bool node = lane < ni;
        const int pnext = wv_pull(pos_o, lane < 63 ? lane + 1 : 63);
        const int dep = node ? np_lca_depth(n, pos_o, pnext) : 0x3fffffff;
        // nearest strictly shallower node on each side (-1: none), visiting the depths in
        // increasing order.  A dense span (the usual case: the depths of one summation tree over a
        // few thousand slots) steps d by one with one ballot each; a wide span (a union of ~1.8 M
        // slots or more) visits only the depths present, the next one by a wave minimum -- at
        // most ni <= 63 of them -- so the record is the LDS kernel's for any union size
        int nl = -1, nr = -1;
        const int dlo = wv_min(dep), dhi = wv_max(node ? dep : -1);
        const bool dense = dhi - dlo < 4 * kMaxLevels;
        {
            uint64_t sh = 0;                                       // nodes shallower than d
            for (int d = dlo; d <= dhi;) {
                const bool at = node && dep == d;
                const uint64_t e = __ballot(at);
                if (e != 0) {
                    if (at) {
                        const uint64_t lm = sh & below, rm = sh & above;
                        nl = lm ? 63 - __builtin_clzll(lm) : -1;
                        nr = rm ? __builtin_ctzll(rm) : -1;
                    }
                    sh |= e;
                }
                d = dense ? d + 1 : wv_min(node && dep > d ? dep : 0x7fffffff);
            }
        }
        // parent = the deeper of the two; a node is its parent's left child when the parent is on
        // its right.  Children go to the parent's lane (id + 1; 0 = none -- a term child); the
        // other lanes push to lane 63, never a node (ni <= 63)
        const int dl = wv_pull(dep, nl < 0 ? 0 : nl), dr = wv_pull(dep, nr < 0 ? 0 : nr);
        const int par = nl < 0 ? nr : nr < 0 ? nl : (dl > dr ? nl : nr);
        const bool lchild = node && par >= 0 && par == nr, rchild = node && par >= 0 && par == nl;
        const int lcn = wv_push(lane + 1, lchild ? par : 63);
        const int rcn = wv_push(lane + 1, rchild ? par : 63);
        // child ids: term t -> t, node kk -> m + kk
        const int lch = lcn ? m + lcn - 1 : lane, rch = rcn ? m + rcn - 1 : lane + 1;
        // heights (the DAG level of an add: 1 + its children's), relaxed until they settle
        int h = node ? 1 : 0;
        for (int it = 0; it < ni + 1; ++it) {
            const int ha = wv_pull(h, lch < m ? 0 : lch - m), hb = wv_pull(h, rch < m ? 0 : rch - m);
            const int ca = lch < m ? 0 : ha, cb = rch < m ? 0 : hb;
            const int hn = node ? (ca > cb ? ca : cb) + 1 : 0;
            const bool ch = hn != h;
            h = hn;
            if (__ballot(ch) == 0ull) break;
        }
        const int L = wv_max(h);
        if (L > kMaxLevels) {       // deeper than the record's level table (turnover_terms_kernel)
            if (lane == 0) {
                R[0] = -2;
                R[1] = 0;
                R[2] = 0;
                R[3] = 0;
                rlen[i] = 4;
            }
            continue;
        }
        // level order: the nodes of lower levels first, node order inside a level; lane l < L
        // holds the cumulative end of level l + 1
        int nid = 0, lend = 0, base = 0;
        for (int l = 1; l <= L; ++l) {
            const bool at = node && h == l;
            const uint64_t e = __ballot(at);
            if (at) nid = base + __popcll(e & below);
            base += __popcll(e);
            if (lane == l - 1) lend = base;
        }
        // (the pulls run on every lane: a ds_bpermute reads 0 from a lane the EXEC mask disables)
        const int ida = wv_pull(nid, lch < m ? 0 : lch - m), idb = wv_pull(nid, rch < m ? 0 : rch - m);
        const int na = lch < m ? lch : m + ida;
        const int nb = rch < m ? rch : m + idb;
        if (lane == 0) {
            R[0] = m;
            R[1] = ni;
            R[2] = L;
            R[3] = 0;
            rlen[i] = 4 + m + ni + L;
        }
        if (lane < m) R[4 + lane] = code_o;
        if (node) R[4 + m + nid] = na | (nb << 16);
        if (lane < L) R[4 + m + ni + lane] = lend;
    }
}

// staging of the scan: dates per chunk and record words per buffer.  The single sequence (the
// headline) stages 64 dates in 156 KB of LDS; a bootstrap path (config E: 1,024 workgroups) stages
// 8 in 31 KB, so five paths share a CU and all of them run in one round (round 5: 156 KB kept one
// path per CU, four rounds).  A buffer holds at least one record (kRec words).
constexpr int kChunkDates = 64;
constexpr int kBufWords = 12288;
constexpr int kPathChunkDates = 8;
constexpr int kPathBufWords = 2048;

// x / d from r = RN(1 / d) (Markstein: q0 = RN(x r), e = fma(-q0, d, x), q = RN(q0 + e r) is the
// IEEE quotient when r is the correctly rounded reciprocal and nothing under- or overflows; the
// same correction as lasso.hip div_r).  Out of that range (or d = 0, inf, NaN) the IEEE division.
__device__ __forceinline__ double mdiv(double x, double d, double r) {
    const double q0 = x * r;
    const double e = __builtin_fma(-q0, d, x);
    const double q1 = __builtin_fma(e, r, q0);
    const double aq = __builtin_fabs(q0), ar = __builtin_fabs(r);
    const bool ok = aq > 0x1p-400 && aq < 0x1p400 && ar > 0x1p-400 && ar < 0x1p400;
    if (__builtin_expect(!ok, 0)) return x / d;
    return q1;
}

// One workgroup of 2 waves.  Wave 1 stages chunk c+1 (records, sums and the reciprocals of the
// two price sums) into LDS while wave 0 runs chunk c; one barrier per chunk.  Wave 0 keeps V /
// V_prev replicated in every lane; its per-date chain (round 4: 1.95 -> ~0.5 us per date) is
//   V -> share counts (Markstein quotients on the staged reciprocals, 3 dependent ops each)
//     -> the |c - n| leaves -> the DAG levels of the turnover sum -> turnover cost / V
//     (Markstein on RN(1 / V), computed beside the tree) -> V (1 + daily);
// every V-independent read of date j + 1 (record header, leaf codes, sums, reciprocals, the
// first level's add descriptor) is issued during date j, and the DAG levels run without
// lgkmcnt(0) waits: only this wave touches node[], and one wave's LDS operations execute in
// order, so a level's reads see the previous level's writes.
// Workgroup b scans the steps [b * nd, (b + 1) * nd) (bootstrap path b; one workgroup for the
// plain sequence); the sums of step i are those of book slot ix(i).
template <int kChunkDates, int kBufWords>
__global__ __launch_bounds__(128) void pnl_scan_kernel(int64_t nd, const double* sums,
                                                      const int32_t* rec, const int32_t* rlen,
                                                      double v0, double rate, double* value,
                                                      double* turnover, double* long_ret,
                                                      double* short_ret, const int32_t* idx) {
    AFM_SCAN_PRIO_SET();
    __shared__ int buf[2][kBufWords];
    __shared__ double sm[2][kChunkDates + 1][4];
    __shared__ double rcp[2][kChunkDates + 1][2];           // RN(1 / S[2]), RN(1 / S[3])
    __shared__ int64_t cstart[2];
    __shared__ int ccount[2];
    __shared__ double node[2 * kMaxTerms];
    // per staged date, derived by the loader from its record: {offset, m, nint, L}, each lane's
    // leaf code (lanes < m) and dataflow descriptor (lanes < nint) -- so the scan reads a date's
    // inputs with independent loads (one LDS round trip) instead of a chain through the record
    __shared__ int4 hdr[2][kChunkDates];
    __shared__ unsigned char code8[2][kChunkDates][64];
    __shared__ unsigned gdv[2][kChunkDates][64];
    // two-level dataflow (DAGs of <= 64 adds): lane q's grandchildren ids, 8 bits each (ids <=
    // 129 there); a leaf child c reads as (c, kZ), node[kZ] = -0.0, the exact additive identity
    // (x + -0 = x for every x, +0 and -0 included)
    constexpr int kZ = 255;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t base = (int64_t)blockIdx.x * nd;
    rec += base * kRec;
    rlen += base;
    if (idx) idx += base;
    value += (int64_t)blockIdx.x * (nd + 1);
    turnover += base;
    long_ret += base;
    short_ret += base;

    // loader (wave 1): stage the dates [i0, i0 + c) into buffer b; returns i0 + c
    auto stage = [&](int64_t i0, int b) -> int64_t {
        int len = 0;
        if (i0 + lane < nd) len = rlen[i0 + lane];
        int incl = len;                                            // wave inclusive scan
        for (int o = 1; o < 64; o <<= 1) {
            const int x = __shfl_up(incl, o, 64);
            if (lane >= o) incl += x;
        }
        static_assert(kBufWords >= kRec && kChunkDates <= 64, "a chunk holds 1..64 records");
        const bool fits = (i0 + lane < nd) && lane < kChunkDates && incl <= kBufWords;
        const u64 fm = __ballot(fits);
        const int c = fm == ~0ull ? 64 : __builtin_ctzll(~fm);   // prefix of dates that fits
        // the records' first 128 words for 16 dates at a time, every load issued before the LDS
        // writes (round 4: a date-by-date copy waited one global-load latency per date, ~1 us,
        // and the scan waited for it at the chunk barrier); longer records' tails after
        constexpr int kB = 16;
        for (int j0 = 0; j0 < c; j0 += kB) {
            int v0[kB], v1[kB];
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                const int j = j0 + u < c ? j0 + u : c - 1;
                const int l = __shfl(len, j, 64);
                const int32_t* src = rec + (i0 + j) * kRec;
                v0[u] = lane < l ? src[lane] : 0;
                v1[u] = lane + 64 < l ? src[lane + 64] : 0;
            }
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                const int j = j0 + u < c ? j0 + u : c - 1;
                const int o = __shfl(incl - len, j, 64), l = __shfl(len, j, 64);
                if (j0 + u < c) {
                    if (lane < l) buf[b][o + lane] = v0[u];
                    if (lane + 64 < l) buf[b][o + lane + 64] = v1[u];
                }
            }
        }
        for (int j = 0; j < c; ++j) {
            const int o = __shfl(incl - len, j, 64), l = __shfl(len, j, 64);
            if (l <= 128) continue;                                  // (uniform)
            const int32_t* src = rec + (i0 + j) * kRec;
            for (int e = 128 + lane; e < l; e += 64) buf[b][o + e] = src[e];
        }
        for (int j = 0; j < c; ++j) {            // (this wave's own LDS writes: in order)
            const int o = __shfl(incl - len, j, 64);
            const int* R = &buf[b][o];
            const int m = R[0], nint = R[1], L = R[2];
            code8[b][j][lane] = (unsigned char)(lane < m ? R[4 + lane] : 0);
            unsigned g = 0u;
            if (m > 0 && nint <= 64 && lane < nint) {
                const int wd = R[4 + m + lane], c0 = wd & 0xffff, c1 = wd >> 16;
                const int ga = c0 >= m ? R[4 + c0] : (c0 | (kZ << 16));
                const int gb = c1 >= m ? R[4 + c1] : (c1 | (kZ << 16));
                g = (unsigned)(ga & 0xff) | (unsigned)((ga >> 16) & 0xff) << 8 |
                    (unsigned)(gb & 0xff) << 16 | (unsigned)((gb >> 16) & 0xff) << 24;
            }
            gdv[b][j][lane] = g;
            if (lane == 0) hdr[b][j] = make_int4(o, m, nint, L);
        }
        constexpr int kSumIt = ((kChunkDates + 1) * 4 + 63) / 64;   // all loads first
        double sv[kSumIt];
#pragma unroll
        for (int u = 0; u < kSumIt; ++u) {
            const int e = lane + 64 * u;
            const int64_t ii = i0 - 1 + e / 4;
            sv[u] = e < (c + 1) * 4 && ii >= 0 ? sums[(idx ? (int64_t)idx[ii] : ii) * 4 + e % 4] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kSumIt; ++u) {
            const int e = lane + 64 * u;
            if (e < (c + 1) * 4) {
                sm[b][e / 4][e % 4] = sv[u];
                if (e % 4 >= 2) rcp[b][e / 4][e % 4 - 2] = 1.0 / sv[u];
            }
        }
        if (lane == 0) { cstart[b] = i0; ccount[b] = c; }
        return i0 + c;
    };

    int64_t next = 0;
    if (wave == 1) next = stage(0, 0);
    __syncthreads();
    double V = v0;
    // share counts of the previous date, (V_prev / 2) / price sums: the same quotients the
    // previous date computed as its new ones, carried instead of divided again
    double qa = 0.0, qb = 0.0;
    if (wave == 0 && lane == 0) value[0] = v0;
    for (int ch = 0;; ++ch) {
        const int b = ch & 1;
        const int c = ccount[b];
        if (c == 0) break;                                        // uniform (read after barrier)
        if (wave == 1) {
            if (next < nd) next = stage(next, b ^ 1);
            else if (lane == 0) ccount[b ^ 1] = 0;
        } else {
            const int64_t i0 = cstart[b];
            // date j's V-independent inputs, read one date ahead
            struct Pre {
                const int* R;
                int m, nint, L, code;
                unsigned gd;
                double s0, s1, s2, s3, r2, r3;
            };
            auto prefetch = [&](int j) {         // independent loads only (see hdr)
                Pre f;
                const int4 hd = hdr[b][j];
                f.R = &buf[b][hd.x];
                f.m = hd.y;
                f.nint = hd.z;
                f.L = hd.w;
                const double* S = sm[b][j + 1];
                f.s0 = S[0]; f.s1 = S[1]; f.s2 = S[2]; f.s3 = S[3];
                f.r2 = rcp[b][j + 1][0];
                f.r3 = rcp[b][j + 1][1];
                f.code = code8[b][j][lane];
                // the dataflow evaluation's grandchildren (internal node `lane`, level order)
                f.gd = gdv[b][j][lane];
                return f;
            };
            Pre cur = prefetch(0);
            for (int j = 0; j < c; ++j) {
                const Pre f = cur;
                if (j + 1 < c) cur = prefetch(j + 1);
                const int m = f.m;
                double to = 0.0;
                const double size = V / 2;
                const double qc = mdiv(size, f.s2, f.r2), qd = mdiv(size, f.s3, f.r3);
                const double rv = 1.0 / V;                             // beside the tree
                if (m == -2) to = __builtin_nan("");   // turnover DAG deeper than kMaxLevels
                if (m > 0) {
                    const int* R = f.R;
                    const int nint = f.nint, L = f.L;
                    auto leaf = [&](int sd) {
                        const int ps = sd / 3, ns = sd % 3;
                        // (-x) / y == -(x / y) exactly: the reference's -size / sum
                        const double cv = ps == 0 ? qa : (ps == 1 ? -qb : 0.0);
                        const double nv = ns == 0 ? qc : (ns == 1 ? -qd : 0.0);
                        const double d = cv - nv;
                        return d < 0 ? -d : d;
                    };
                    if (lane < m) node[lane] = leaf(f.code);
                    for (int e = lane + 64; e < m; e += 64) node[e] = leaf(R[4 + e]);
                    if (nint <= 64 && nint > 0) {
                        // dataflow: lane q recomputes internal node q from its grandchildren's
                        // current values, (gaa + gab) + (gba + gbb) -- the additions its children's
                        // lanes make -- ceil(L / 2) times (a node of height h is final after
                        // ceil(h / 2) passes); the root stays in its lane's register
                        const int aa = f.gd & 0xff, ab = (f.gd >> 8) & 0xff;
                        const int ba = (f.gd >> 16) & 0xff, bb = f.gd >> 24;
                        if (lane == 0) node[kZ] = -0.0;      // (the level path may reuse it)
                        double v = 0.0;
                        for (int l = 0; l < L; l += 2) {
                            v = (node[aa] + node[ab]) + (node[ba] + node[bb]);
                            if (lane < nint) node[m + lane] = v;
                        }
                        const uint64_t rb = __builtin_bit_cast(uint64_t, v);
                        const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)rb, nint - 1);
                        const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(rb >> 32), nint - 1);
                        to = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo) / 2;
                    } else {                          // the level-by-level path
                        const int* adds = R + 4 + m;
                        const int* lend = adds + nint;
                        // one DAG level per step, no lgkmcnt(0) wait (see above); the next level's
                        // first add descriptor is fetched while this level's node reads are in flight
                        int st = 0;
                        int en = L > 0 ? lend[0] : 0;
                        int wcur = lane < en ? adds[lane] : 0;
                        for (int l = 0; l < L; ++l) {
                            const int en2 = l + 1 < L ? lend[l + 1] : en;
                            const int wnext = en + lane < en2 ? adds[en + lane] : 0;
                            for (int e = st + lane; e < en; e += 64) {
                                const int w = e == st + lane ? wcur : adds[e];
                                node[m + e] = node[w & 0xffff] + node[w >> 16];
                            }
                            st = en;
                            en = en2;
                            wcur = wnext;
                        }
                        to = node[nint > 0 ? m + nint - 1 : 0] / 2;
                    }
                }
                double daily = (f.s0 - f.s1) / 2;
                daily -= mdiv(to * rate, V, rv);
                const double Vn = V * (1 + daily);
                if (lane == 0) {
                    const int64_t i = i0 + j;
                    long_ret[i] = f.s0;
                    short_ret[i] = f.s1;
                    turnover[i] = to;
                    value[i + 1] = Vn;
                }
                qa = qc;
                qb = qd;
                V = Vn;
            }
        }
        __syncthreads();
    }
}

// ---- bootstrap paths (BASELINE config E) ------------------------------------------------------
// A path is a sequence of rebalance-date slots drawn with replacement; each step re-runs the
// calculate_portfolio update of KKT:842-892 on the slot's date.  Books, weights and PnL sums are
// per date (path-independent) and come from rebalance_kernel; only the turnover alignment --
// the union of the previous and the current step's prediction sets (KKT:839) -- and the value
// recursion depend on the path.

// pbits[d][w] = prediction presence (non-NaN) of the assets 64w .. 64w+63 on rebalance slot d.
// One wave per (slot, word): a ballot over a coalesced 512-B row segment.
__global__ __launch_bounds__(256) void pred_bits_kernel(int64_t lda, const int32_t* dates,
                                                       int64_t nd, const double* pred,
                                                       uint64_t* pbits) {
    const int64_t nw = lda >> 6;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t d = blockIdx.y;
    if (w >= nw) return;
    const double v = pred[(int64_t)dates[d] * lda + w * 64 + (threadIdx.x & 63)];
    const u64 b = __ballot(v == v);
    if ((threadIdx.x & 63) == 0) pbits[d * nw + w] = b;
}

// One wave per step i (> 0 within its path): union U = P(prev) | P(cur) word by word, a wave
// prefix scan of the popcounts, then the union position of every book member that is also
// predicted on the other step (the pair enters the turnover; others align with NaN and drop).
// Writes upos[i][side][0][*] (current members), upos[i-1][side][1][*] (previous members) and
// usize[i][0] = |U| -- the layout turnover_terms_kernel reads.
__global__ __launch_bounds__(64) void pair_union_kernel(int64_t steps, const int32_t* path,
                                                       int64_t nw, const uint64_t* pbits,
                                                       const int32_t* k_out,
                                                       const int32_t* books, int32_t* upos,
                                                       int64_t* usize) {
    __shared__ int prefix[kMaxWords];
    const int64_t i = blockIdx.x;
    const int lane = threadIdx.x;
    if (i % steps == 0) {
        if (lane == 0) usize[i * 2] = 0;
        return;
    }
    const int64_t dp = path[i - 1], dc = path[i];
    const uint64_t* Pp = pbits + dp * nw;
    const uint64_t* Pc = pbits + dc * nw;
    int carry = 0;
    for (int64_t w0 = 0; w0 < nw; w0 += 64) {
        const int64_t w = w0 + lane;
        const int c = w < nw ? __popcll(Pp[w] | Pc[w]) : 0;
        int incl = c;
        for (int o = 1; o < 64; o <<= 1) {
            const int x = __shfl_up(incl, o, 64);
            if (lane >= o) incl += x;
        }
        if (w < nw) prefix[w] = carry + incl - c;
        carry += __shfl(incl, 63, 64);
    }
    __syncthreads();
    if (lane == 0) usize[i * 2] = carry;
    auto pos_of = [&](int a, const uint64_t* other) -> int {
        const int wa = a >> 6, ba = a & 63;
        if (!((other[wa] >> ba) & 1ull)) return -1;
        const u64 lowm = ba ? ((1ull << ba) - 1ull) : 0ull;
        return prefix[wa] + __popcll((Pp[wa] | Pc[wa]) & lowm);
    };
    const int kp = k_out[dp], k = k_out[dc];
    for (int e = lane; e < 2 * kp; e += 64) {
        const int side = e / kp, q = e % kp;
        upos[(((i - 1) * 2 + side) * 2 + 1) * kMaxK + q] = pos_of(books[(dp * 2 + side) * kMaxK + q], Pc);
    }
    for (int e = lane; e < 2 * k; e += 64) {
        const int side = e / k, q = e % k;
        upos[((i * 2 + side) * 2 + 0) * kMaxK + q] = pos_of(books[(dc * 2 + side) * kMaxK + q], Pp);
    }
}

}  // namespace
}  // namespace afm

using namespace afm;

// history rows [t0, t0 + n) of the [T][lda] panel -> member-major [lda][n], NaN where the
// presence bit is clear (books over 32 names stage their windows from it, coalesced)
// dates / window (window > 0): only the 64-date tiles that meet the rebalance dates' windows,
// [dates[0] - window, dates[nd - 1] + 1), are copied (the dates ascend); the rest of hT is never
// read (the whole panel was transposed on every call)
__global__ __launch_bounds__(256) void hist_transpose_kernel(int64_t lda, int64_t A,
                                                             const double* hist,
                                                             const uint64_t* hbits, int64_t t0,
                                                             int64_t n, double* hT,
                                                             const int32_t* dates, int64_t nd,
                                                             int64_t window) {
    __shared__ double tile[64][65];
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const int64_t tb = (int64_t)blockIdx.x * 64, ab = (int64_t)blockIdx.y * 64;
    if (window > 0) {
        const int64_t lo = (int64_t)dates[0] - window, hi = (int64_t)dates[nd - 1] + 1;
        if (t0 + tb + 64 <= lo || t0 + tb >= hi) return;          // uniform: the whole tile
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int rr = w + 4 * j;
        const int64_t t = t0 + tb + rr, a = ab + l;
        double v = __builtin_nan("");
        if (tb + rr < n && a < A) {
            const u64 wb = hbits[(t >> 6) * lda + a];
            const double x = hist[t * lda + a];
            v = (wb >> (t & 63)) & 1ull ? x : v;
        }
        tile[rr][l] = v;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int c = w + 4 * j;
        if (tb + l < n) hT[(ab + c) * n + tb + l] = tile[l][c];
    }
}

// the turnover DAG records of n steps: the one-wave kernel for the steps with books of <= kWaveK
// names, the persistent LDS kernel for the steps it lists in rest (n + 1 words of scratch)
static hipError_t launch_turnover_terms(afm_ctx* ctx, int64_t n, const int32_t* k_out,
                                        const int32_t* books, const int32_t* upos,
                                        const int64_t* usize, int32_t* rec, int32_t* rlen,
                                        const int32_t* idx, int64_t seq, int32_t* rest) {
    const int64_t ncu = afm_ctx_cus(ctx);
    hipError_t e = hipMemsetAsync(rest, 0, sizeof(int32_t), ctx->stream);
    if (e != hipSuccess) return e;
    const int64_t gw = std::min<int64_t>((n + 3) / 4, 8 * ncu);           // 4 waves per workgroup
    hipLaunchKernelGGL(turnover_terms_wave_kernel, dim3((unsigned)gw), dim3(256), 0, ctx->stream, n,
                       k_out, books, upos, usize, rec, rlen, idx, seq, rest);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int64_t gl = std::min<int64_t>(n, 4 * ncu);
    hipLaunchKernelGGL(turnover_terms_kernel, dim3((unsigned)gl), dim3(64), 0, ctx->stream, n, k_out,
                       books, upos, usize, rec, rlen, idx, seq, (const int32_t*)rest);
    return hipGetLastError();
}

template <int KM>
static int launch_rebalance(afm_ctx* ctx, const RebArgs& r) {
    const size_t smem = sizeof(Shared<KM>);
    AFM_HIP(afm_lds_opt_in(ctx, (const void*)rebalance_kernel<KM>, (int)smem));
    hipLaunchKernelGGL(rebalance_kernel<KM>, dim3((unsigned)r.nd, 2), dim3(kT), smem, ctx->stream,
                       r);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

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
    AFM_CHECK_ARG(top_n >= 0 && top_n <= kMaxK, "top_n must be in [0, 128]");
    AFM_CHECK_ARG(dates && pred && trad_bits && hist && hist_bits && close && tmr && k_out &&
                      books && weights && sums && upos && usize && status, "null buffer");
    AFM_CHECK_ARG(lo <= hi, "lo > hi");
    if (nd <= 0) return AFM_OK;
    AFM_HIP(hipMemsetAsync(status, 0, sizeof(int32_t) * (size_t)nd, ctx->stream));
    // books of more than one pass of member pairs re-stage their history once per pass: give
    // them a contiguous copy of their window
    const int64_t hrows = window > 0 ? window : (h_t1 > h_t0 ? h_t1 - h_t0 : 0);
    AFM_CHECK_ARG((int64_t)top_n * hrows < (int64_t)1 << 31, "top_n x history rows over 2^31");
    double* hscr = nullptr;
    double* histT = nullptr;
    int64_t hT0 = 0, hTn = 0;
    if (top_n > 32) {
        // books over 32 names: the history panel member-major once, instead of a strided gather
        // per book (each member's window then one contiguous run)
        hT0 = window > 0 ? 0 : h_t0;
        hTn = window > 0 ? T : (h_t1 > h_t0 ? h_t1 - h_t0 : 0);
        if (hTn > 0) {
            hipError_t e;
            histT = (double*)afm_ctx_scratch(ctx, AFM_SCRATCH_REB_HIST,
                                             sizeof(double) * (size_t)lda * hTn, &e);
            AFM_HIP(e);
            hipLaunchKernelGGL(hist_transpose_kernel, dim3((unsigned)((hTn + 63) / 64),
                                                           (unsigned)(lda / 64)),
                               dim3(256), 0, ctx->stream, lda, A, hist, hist_bits, hT0, hTn, histT,
                               dates, nd, window);
            AFM_HIP(hipGetLastError());
        }
    } else if (top_n * (top_n + 1) / 2 > kT && hrows > 0) {
        hipError_t e;
        hscr = (double*)afm_ctx_scratch(ctx, AFM_SCRATCH_REB_SCR,
                                        sizeof(double) * (size_t)nd * 2 * top_n * hrows, &e);
        AFM_HIP(e);
    }
    RebArgs r{T, lda, A, dates, nd, pred, trad_bits, hist, hist_bits, h_t0, h_t1, window, close,
              tmr, top_n, lo, hi, hscr, histT, hT0, hTn, hrows, 0, nullptr, k_out, books, weights,
              sums, upos, usize, status};
#ifdef AFM_PROBE                     // profiling build (make prof): phase experiments
    if (const char* e = getenv("AFM_REB_PROBE")) r.probe = atoi(e);
#endif
    if (r.probe & 4) AFM_HIP(hipMallocAsync((void**)&r.stamps, sizeof(int64_t) * nd * 16, ctx->stream));
    const int rc = top_n <= 32 ? launch_rebalance<32>(ctx, r) : launch_rebalance<kMaxK>(ctx, r);
    if (r.stamps) {                  // experiment: mean phase durations per workgroup
        std::vector<int64_t> h((size_t)nd * 16);
        AFM_HIP(hipMemcpyAsync(h.data(), r.stamps, sizeof(int64_t) * nd * 16, hipMemcpyDeviceToHost,
                               ctx->stream));
        AFM_HIP(hipStreamSynchronize(ctx->stream));
        double acc[7] = {0, 0, 0, 0, 0, 0, 0};
        for (int64_t b = 0; b < nd * 2; ++b) {
            const int64_t* x = &h[b * 8];
            for (int j = 0; j < 4; ++j) acc[j] += (double)(x[j + 1] - x[j]);
            acc[4] += (double)(x[5] - x[1]);
            acc[5] += (double)(x[6] - x[2]);
            acc[6] += (double)x[7];
        }
        const double f = 1.0 / (nd * 2 * 100.0);
        fprintf(stderr, "rebalance phases (us/workgroup, 100 MHz clock): select %.1f cov %.1f "
                "(gather %.1f) qp %.1f (setup %.1f, %.1f iterations) out %.1f\n", acc[0] * f,
                acc[1] * f, acc[4] * f, acc[2] * f, acc[5] * f, acc[6] / (nd * 2), acc[3] * f);
        AFM_HIP(hipFree(r.stamps));
    }
    return rc;
}

extern "C" int afm_pnl_scan_f64(afm_ctx* ctx, int64_t nd, const int32_t* k_out,
                                const int32_t* books, const double* sums, const int32_t* upos,
                                const int64_t* usize, double v0, double rate, double* value,
                                double* turnover, double* long_ret, double* short_ret) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(k_out && books && sums && upos && usize && value && turnover && long_ret &&
                      short_ret, "null buffer");
    if (nd <= 0) return AFM_OK;
    AFM_CHECK_ARG(nd <= 0x7fffffff, "nd too large for one launch");
    hipError_t e;
    int32_t* work = (int32_t*)afm_ctx_scratch(ctx, AFM_SCRATCH_PNL,
                                              sizeof(int32_t) * ((size_t)nd * (kRec + 2) + 1), &e);
    AFM_HIP(e);
    int32_t* rec = work;
    int32_t* rlen = work + nd * kRec;
    AFM_HIP(launch_turnover_terms(ctx, nd, k_out, books, upos, usize, rec, rlen, nullptr, nd,
                                  rlen + nd));
    hipLaunchKernelGGL((pnl_scan_kernel<kChunkDates, kBufWords>), dim3(1), dim3(128), 0, ctx->stream,
                       nd, sums, rec, rlen, v0,
                       rate, value, turnover, long_ret, short_ret, (const int32_t*)nullptr);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_min_variance_weights_f64(afm_ctx* ctx, const double* R, int64_t rows,
                                            int64_t ld, int k, double lo, double hi, double* w,
                                            double* cov, int32_t* status) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(k >= 1 && k <= kMaxK && ld >= k && rows >= 0, "need 1 <= k <= 128, ld >= k");
    AFM_CHECK_ARG(R && w && cov && status && lo <= hi, "bad arguments");
    const size_t smem = sizeof(Shared<kMaxK>);
    AFM_HIP(afm_lds_opt_in(ctx, (const void*)weights_kernel, (int)smem));
    hipLaunchKernelGGL(weights_kernel, dim3(1), dim3(kT), smem, ctx->stream, R, rows, ld, k, lo,
                       hi, w, cov, status);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_bootstrap_pnl_f64(afm_ctx* ctx, int64_t lda, const int32_t* dates, int64_t nd,
                                     const double* pred, const int32_t* k_out,
                                     const int32_t* books, const double* sums, int64_t npaths,
                                     int64_t steps, const int32_t* path, double v0, double rate,
                                     double* value, double* turnover, double* long_ret,
                                     double* short_ret) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(dates && pred && k_out && books && sums && path && value && turnover &&
                      long_ret && short_ret, "null buffer");
    AFM_CHECK_ARG(lda > 0 && lda % 64 == 0 && lda / 64 <= kMaxWords, "bad lda (max 32768 assets)");
    AFM_CHECK_ARG(nd > 0 && npaths >= 0 && steps >= 0 && npaths <= 0x7fffffff, "bad sizes");
    const int64_t n = npaths * steps;
    if (n == 0) return AFM_OK;
    AFM_CHECK_ARG(n <= 0x7fffffff, "npaths * steps too large for one launch");
    const int64_t nw = lda / 64;
    // scratch: pbits [nd][nw] u64, upos [n][2][2][kMaxK], usize [n][2], rec [n][kRec], rlen [n],
    // rest [n + 1]
    const size_t b_pb = sizeof(uint64_t) * nd * nw, b_up = sizeof(int32_t) * n * 4 * kMaxK,
                 b_us = sizeof(int64_t) * n * 2, b_rec = sizeof(int32_t) * (n * (kRec + 2) + 1);
    hipError_t e;
    char* work = (char*)afm_ctx_scratch(ctx, AFM_SCRATCH_BOOT, b_pb + b_up + b_us + b_rec, &e);
    AFM_HIP(e);
    uint64_t* pbits = (uint64_t*)work;
    int64_t* usize = (int64_t*)(work + b_pb);
    int32_t* upos = (int32_t*)(work + b_pb + b_us);
    int32_t* rec = (int32_t*)(work + b_pb + b_us + b_up);
    int32_t* rlen = rec + n * kRec;
    hipLaunchKernelGGL(pred_bits_kernel, dim3((unsigned)((nw + 3) / 4), (unsigned)nd), dim3(256),
                       0, ctx->stream, lda, dates, nd, pred, pbits);
    AFM_HIP(hipGetLastError());
    hipLaunchKernelGGL(pair_union_kernel, dim3((unsigned)n), dim3(64), 0, ctx->stream, steps,
                       path, nw, pbits, k_out, books, upos, usize);
    AFM_HIP(hipGetLastError());
    AFM_HIP(launch_turnover_terms(ctx, n, k_out, books, upos, usize, rec, rlen, path, steps,
                                  rlen + n));
    hipLaunchKernelGGL((pnl_scan_kernel<kPathChunkDates, kPathBufWords>), dim3((unsigned)npaths),
                       dim3(128), 0, ctx->stream, steps,
                       sums, rec, rlen, v0, rate, value, turnover, long_ret, short_ret, path);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

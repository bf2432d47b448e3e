// Signal evaluation: AlphaSignalAnalyzer.run() without plotting
// ("KKT Yuliang Jiang.py":298-375), on calendar grids, bit-exact with pandas 2.3.3.
//
//  fwd_returns_kernel   A1  k-th next present price row per asset (k = 1, 2, 5): c'/c - 1, kept
//                           when <= 1 (KKT:311-312); one thread per cell, presence-word scans.
//  xs_prepare_kernel    A1  per date (one workgroup): the merge/dropna cascade of KKT:313 and the
//                           per-date demean of KKT:315-318 -- mean = numpy pairwise sum / n over
//                           the rows surviving each step, evaluated with numpy's exact tree
//                           (leaves in parallel, combine in order); writes the surviving rows
//                           compacted (ascending security id = the reference's row order).
//  xs_rank_kernel       A3/A4 per date: exact ranks (method='first': ties by row position),
//                           ascending and descending, from 2048-row LDS bitonic-sorted chunks +
//                           binary-search merge counts.
//  xs_stats_kernel      A2-A4 one workgroup per date, rows staged through LDS; in lanes: pandas
//                           nancorr Welford IC (return = the later column), Kahan group means per
//                           decile layer (layer = int(rank/n*10)+1, KKT:328-330), factor-weighted
//                           top-10 returns summed in the string-sorted pivot column order
//                           (KKT:362-369).
//  xs_series_kernel     A2-A4 cumulative layer / long-short / top-k series and the per-year IR
//                           (pairwise mean / two-pass std of the IC values, KKT:353).
#include "afm_internal.h"

#include <algorithm>
#include <vector>

#pragma clang fp contract(off)

namespace afm {
namespace {

typedef unsigned long long u64;
constexpr int kT = 256;
constexpr int kWT = 1024;              // per-date analyzer kernels: 16 waves (latency hiding)
constexpr int kChunk = 2048;          // rows per LDS-sorted chunk
constexpr int kMaxLeaves = 1024;      // pairwise leaves (n <= 65536)
constexpr int kTopK = 10;
constexpr int kLayers = 10;

__device__ __forceinline__ double qnan() { return __builtin_nan(""); }
__device__ __forceinline__ bool bit_at(const uint64_t* bits, int64_t lda, int64_t t, int64_t a) {
    return (bits[(t >> 6) * lda + a] >> (t & 63)) & 1ull;
}
__device__ __forceinline__ u64 okey(double v) {
    if (v == 0.0) v = 0.0;
    u64 u = (u64)__double_as_longlong(v);
    return (u >> 63) ? ~u : (u | (1ull << 63));
}

// ---- A1: forward returns -------------------------------------------------------------------
__global__ __launch_bounds__(256) void fwd_returns_kernel(int64_t T, int64_t lda,
                                                          const double* close,
                                                          const uint64_t* pbits, double* fr) {
    const int64_t a = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    const int64_t t = (int64_t)blockIdx.y * 4 + (threadIdx.x >> 6);
    if (t >= T) return;
    const int64_t plane = T * lda;
    const int64_t cell = t * lda + a;
    double r[3] = {qnan(), qnan(), qnan()};
    if (bit_at(pbits, lda, t, a)) {
        const int ks[3] = {1, 2, 5};
        const int64_t nch = (T + 63) / 64;
        int64_t ch = t >> 6;
        const int s = (int)(t & 63);
        u64 w = pbits[ch * lda + a];
        u64 rest = (s == 63) ? 0ull : (w >> (s + 1)) << (s + 1);
        int found = 0;
        int64_t nxt[5];
        while (found < 5) {
            while (rest && found < 5) {
                nxt[found++] = ch * 64 + __builtin_ctzll(rest);
                rest &= rest - 1;
            }
            if (found >= 5 || ++ch >= nch) break;
            rest = pbits[ch * lda + a];
        }
        const double c0 = close[cell];
        for (int q = 0; q < 3; ++q) {
            if (found >= ks[q]) {
                double v = close[nxt[ks[q] - 1] * lda + a] / c0 - 1;
                r[q] = (v <= 1) ? v : qnan();       // return_data[return_data[i] <= 1]
            }
        }
    }
    for (int q = 0; q < 3; ++q) fr[q * plane + cell] = r[q];
}

// ---- block helpers ---------------------------------------------------------------------------
// exclusive scan of 0/1 flags over the 256 threads: ballots within the waves, wave totals
// through LDS (two barriers instead of a log-step scan)
template <int NT = kT>
__device__ int block_scan(int v, int* sbuf, int* excl) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u64 m = __ballot(v != 0);
    const int below = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
    if (lane == 0) sbuf[w] = __popcll(m);
    __syncthreads();
    int off = 0, total = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) {
        off += i < w ? sbuf[i] : 0;
        total += sbuf[i];
    }
    __syncthreads();
    *excl = off + below;
    return total;
}

struct PwShared {
    int64_t loff[kMaxLeaves];
    int llen[kMaxLeaves];
    double lval[kMaxLeaves];
    int nleaves;
    int cursor;
    double result;
};

__device__ void pw_enum(PwShared& p, int64_t off, int64_t n) {
    if (n <= 128) {
        p.loff[p.nleaves] = off;
        p.llen[p.nleaves] = (int)n;
        p.nleaves++;
        return;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    pw_enum(p, off, n2);
    pw_enum(p, off + n2, n - n2);
}

__device__ double pw_combine(PwShared& p, int64_t n) {
    if (n <= 128) return p.lval[p.cursor++];
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    double a = pw_combine(p, n2);
    double b = pw_combine(p, n - n2);
    return a + b;
}

__device__ double leaf_sum(const double* a, int n) {
    if (n < 8) {
        double res = 0.;
        for (int i = 0; i < n; ++i) res += a[i];
        return res;
    }
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int i;
    for (i = 8; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
}

// np.add.reduce of v[0..n) -- the identity 0.0, then numpy's pairwise sums of the consecutive
// kNpBuf-element buffers of the ufunc's buffered reduction added one by one (over 8192 elements
// the sum is not one pairwise tree: oracle np_sum, pinned to numpy in tests/test_oracle_golden.py)
// -- evaluated by the whole block
constexpr int64_t kNpBuf = 8192;
template <int NT = kT>
__device__ double block_np_sum(PwShared& p, const double* v, int64_t n) {
    const int tid = threadIdx.x;
    if (tid == 0) {
        p.nleaves = 0;
        p.cursor = 0;
        for (int64_t c0 = 0; c0 < n; c0 += kNpBuf) pw_enum(p, c0, n - c0 < kNpBuf ? n - c0 : kNpBuf);
    }
    __syncthreads();
    for (int l = tid; l < p.nleaves; l += NT) p.lval[l] = leaf_sum(v + p.loff[l], p.llen[l]);
    __syncthreads();
    if (tid == 0) {
        double r = 0.0;
        for (int64_t c0 = 0; c0 < n; c0 += kNpBuf)
            r = r + pw_combine(p, n - c0 < kNpBuf ? n - c0 : kNpBuf);
        p.result = r;
    }
    __syncthreads();
    double r = p.result;
    __syncthreads();
    return r;
}

// ---- A1: per-date merge/dropna cascade + demean --------------------------------------------
struct PrepArgs {
    int64_t T, lda, A;
    const double* sig;        // [T][lda] signal (NaN = no row)
    const double* fr;         // [3][T][lda] forward returns
    double* scratch;          // [T][lda] compaction scratch
    double* rows;             // [4][T][lda]: factor, r1, r2, r5 of surviving rows, compacted
    int32_t* rows_idx;        // [T][lda] asset index of each compacted row
    int32_t* nrows;           // [T] surviving rows per date
    int64_t t0;               // first date processed (workgroup b: date t0 + b)
    int64_t* stamps;          // experiment (AFM_AN_PROBE): 5 phase timestamps per date, or null
    int64_t* clk;             // experiment: shader-clock stamps at phases 0 and 4
};

constexpr int kPT = 256;               // xs_prepare threads (4 waves)
constexpr int kMaxWords = 512;         // A <= 32768
constexpr int kMaxNodes = 1216;        // numpy pairwise-tree nodes of n <= 32768 (leaves >= 57)
constexpr int kMaxLevels = 16;

struct PrepShared {
    u64 mw[3][kMaxWords];              // row masks per step k: signal and returns 1..k present
    int pre[3][kMaxWords + 1];         // exclusive prefix counts of the mask words
    int noff[kMaxNodes], nlen[kMaxNodes], nchild[kMaxNodes];   // one column's tree, level order
    double nval[kMaxNodes];
    int lvl[kMaxLevels + 1];           // level boundaries in the node arrays
    int scan[kPT / 64];
    double mu[3];
};

// One workgroup (4 waves) per date.  The three row masks of KKT:313's merge + dropna steps as
// bit words by ballot over coalesced 64-asset segments, and their prefix counts.  Then per
// return column: its rows compacted (ascending security id) into the scratch row, numpy's
// pairwise summation tree of each 8192-row reduction buffer built level by level (node m > 128
// splits at m/2 - (m/2)%8, as in numpy's pairwise_sum), every leaf summed by its own thread (the
// 8-accumulator block, or the plain loop under 8), the internal nodes added bottom-up level by
// level, the buffers added one by one onto 0.0: mean = sum / n bit-exactly, with no serial
// walk.  Finally the rows surviving all three steps are written compacted with demeaned returns.
__global__ __launch_bounds__(kPT) void xs_prepare_kernel(PrepArgs g) {
    AFM_TAIL_PRIO_SET();
    __shared__ PrepShared sh;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t t = g.t0 + blockIdx.x;
    const int64_t plane = g.T * g.lda;
    const double* sig = g.sig + t * g.lda;
    const double* fr0 = g.fr + t * g.lda;
    double* scr = g.scratch + t * g.lda;
    const int nw = (int)((g.A + 63) / 64);
    if (g.stamps && tid == 0) { g.stamps[t * 5 + 0] = wall_clock64(); g.clk[t * 2] = clock64(); }
    // ---- masks ---------------------------------------------------------------------------
    for (int w0 = wave; w0 < nw; w0 += 16) {
        double v[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t a = (int64_t)(w0 + 4 * u) * 64 + lane;
            const bool in = w0 + 4 * u < nw && a < g.A;
            v[u][0] = in ? sig[a] : qnan();
#pragma unroll
            for (int q = 0; q < 3; ++q) v[u][1 + q] = in ? fr0[q * plane + a] : qnan();
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int w = w0 + 4 * u;
            bool ok = v[u][0] == v[u][0];
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                ok = ok && v[u][1 + q] == v[u][1 + q];
                const u64 m = __ballot(ok);
                if (lane == 0 && w < nw) sh.mw[q][w] = m;
            }
        }
    }
    __syncthreads();
    if (g.stamps && tid == 0) g.stamps[t * 5 + 1] = wall_clock64();
    // ---- prefix counts (wave q scans mask q) -----------------------------------------------
    if (wave < 3) {
        int carry = 0;
        for (int w0 = 0; w0 < nw; w0 += 64) {
            const int w = w0 + lane;
            const int c = w < nw ? __popcll(sh.mw[wave][w]) : 0;
            int incl = c;
            for (int o = 1; o < 64; o <<= 1) {
                const int x = __shfl_up(incl, o, 64);
                if (lane >= o) incl += x;
            }
            if (w < nw) sh.pre[wave][w] = carry + incl - c;
            carry += __shfl(incl, 63, 64);
        }
        if (lane == 0) sh.pre[wave][nw] = carry;
    }
    __syncthreads();
    if (g.stamps && tid == 0) g.stamps[t * 5 + 2] = wall_clock64();
    // ---- per return column: compaction, pairwise tree, mean -------------------------------------
    for (int q = 0; q < 3; ++q) {
        const double* x = fr0 + q * plane;
        const int n = sh.pre[q][nw];
        for (int w = wave; w < nw; w += 4) {
            const u64 m = sh.mw[q][w];
            if ((m >> lane) & 1ull)
                scr[sh.pre[q][w] + __popcll(m & ((1ull << lane) - 1ull))] = x[(int64_t)w * 64 + lane];
        }
        const int nbuf = n > 0 ? (int)((n + kNpBuf - 1) / kNpBuf) : 1;   // level 0: the buffers
        if (tid < nbuf) {
            sh.noff[tid] = (int)(tid * kNpBuf);
            sh.nlen[tid] = n - tid * kNpBuf < kNpBuf ? (int)(n - tid * kNpBuf) : (int)kNpBuf;
        }
        if (tid == 0) {
            sh.lvl[0] = 0;
            sh.lvl[1] = nbuf;
        }
        __syncthreads();
        int nlev = 0;
        for (;;) {                                      // build the levels; sum their leaves
            const int lb = sh.lvl[nlev], le = sh.lvl[nlev + 1];
            if (le == lb) break;                        // (uniform)
            int base = le;
            for (int c0 = lb; c0 < le; c0 += kPT) {
                const int i = c0 + tid;
                const int m = i < le ? sh.nlen[i] : 0;
                const int split = m > 128;
                int ex;
                const int tot = block_scan<kPT>(split, sh.scan, &ex);
                if (i < le) {
                    if (split) {
                        int m2 = m / 2;
                        m2 -= m2 % 8;
                        const int ci = base + 2 * ex;
                        sh.nchild[i] = ci;
                        sh.noff[ci] = sh.noff[i];
                        sh.nlen[ci] = m2;
                        sh.noff[ci + 1] = sh.noff[i] + m2;
                        sh.nlen[ci + 1] = m - m2;
                    } else {
                        sh.nchild[i] = -1;
                        const double* a = scr + sh.noff[i];
                        double res;
                        if (m < 8) {
                            res = 0.;
                            for (int j = 0; j < m; ++j) res += a[j];
                        } else {
                            double r[8];
#pragma unroll
                            for (int j = 0; j < 8; ++j) r[j] = a[j];
                            int j;
                            for (j = 8; j < m - (m % 8); j += 8) {
                                double v8[8];
#pragma unroll
                                for (int u = 0; u < 8; ++u) v8[u] = a[j + u];
#pragma unroll
                                for (int u = 0; u < 8; ++u) r[u] += v8[u];
                            }
                            res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
                            for (; j < m; ++j) res += a[j];
                        }
                        sh.nval[i] = res;
                    }
                }
                base += 2 * tot;
            }
            if (tid == 0) sh.lvl[nlev + 2] = base;
            __syncthreads();
            ++nlev;
        }
        for (int l = nlev - 2; l >= 0; --l) {           // internal nodes, bottom-up
            for (int i = sh.lvl[l] + tid; i < sh.lvl[l + 1]; i += kPT) {
                const int ci = sh.nchild[i];
                if (ci >= 0) sh.nval[i] = sh.nval[ci] + sh.nval[ci + 1];
            }
            __syncthreads();
        }
        if (tid == 0) {                                  // the buffers added one by one
            double r = 0.0;
            for (int c = 0; c < nbuf; ++c) r = r + sh.nval[c];
            sh.mu[q] = n > 0 ? r / (double)n : qnan();
        }
        __syncthreads();
    }
    if (g.stamps && tid == 0) g.stamps[t * 5 + 3] = wall_clock64();
    // ---- surviving rows (all three returns), compacted, returns demeaned ----------------------
    const double mu0 = sh.mu[0], mu1 = sh.mu[1], mu2 = sh.mu[2];
    for (int w = wave; w < nw; w += 4) {
        const u64 m = sh.mw[2][w];
        if (!((m >> lane) & 1ull)) continue;
        const int64_t a = (int64_t)w * 64 + lane;
        const int pos = sh.pre[2][w] + __popcll(m & ((1ull << lane) - 1ull));
        const int64_t o = t * g.lda + pos;
        g.rows[o] = sig[a];
        g.rows[plane + o] = fr0[a] - mu0;
        g.rows[2 * plane + o] = fr0[plane + a] - mu1;
        g.rows[3 * plane + o] = fr0[2 * plane + a] - mu2;
        g.rows_idx[o] = (int32_t)a;
    }
    if (tid == 0) g.nrows[t] = sh.pre[2][nw];
    if (g.stamps && tid == 0) { g.stamps[t * 5 + 4] = wall_clock64(); g.clk[t * 2 + 1] = clock64(); }
}

// ---- A3/A4: exact ranks -------------------------------------------------------------------
struct RankArgs {
    int64_t T, lda;
    const double* rows;       // factor column of the compacted rows
    const int32_t* nrows;
    u64* skey;                // [T][lda] sorted chunk keys
    int32_t* sidx;            // [T][lda] sorted chunk positions
    int32_t* rank_asc;        // [T][lda]
    int32_t* rank_desc;       // [T][lda]
};

__global__ __launch_bounds__(kWT) void xs_rank_kernel(RankArgs g, int lds_rows) {
    // dynamic LDS: phase 1 the sort buffers, phase 2 (n <= lds_rows) the date's sorted chunks
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
    u64* key = reinterpret_cast<u64*>(dyn);
    int32_t* idx = reinterpret_cast<int32_t*>(dyn + sizeof(u64) * kChunk);
    const int tid = threadIdx.x;
    const int64_t t = blockIdx.x;
    const int n = g.nrows[t];
    const int64_t base = t * g.lda;
    const int nch = (n + kChunk - 1) / kChunk;
    for (int c = 0; c < nch; ++c) {
        const int c0 = c * kChunk, len = min(kChunk, n - c0);
        for (int e = tid; e < kChunk; e += kWT) {
            if (e < len) {
                key[e] = okey(g.rows[base + c0 + e]);
                idx[e] = c0 + e;
            } else {
                key[e] = ~0ull;
                idx[e] = 0x7fffffff;
            }
        }
        __syncthreads();
        // bitonic sort of (key, idx) ascending
        for (int size = 2; size <= kChunk; size <<= 1) {
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                for (int e = tid; e < kChunk / 2; e += kWT) {
                    const int lo = 2 * e - (e & (stride - 1));
                    const int hi = lo + stride;
                    const bool up = ((lo & size) == 0);
                    const u64 ka = key[lo], kb = key[hi];
                    const int ia = idx[lo], ib = idx[hi];
                    const bool gt = (ka > kb) || (ka == kb && ia > ib);
                    if (gt == up) {
                        key[lo] = kb; key[hi] = ka;
                        idx[lo] = ib; idx[hi] = ia;
                    }
                }
                __syncthreads();
            }
        }
        for (int e = tid; e < len; e += kWT) {
            g.skey[base + c0 + e] = key[e];
            g.sidx[base + c0 + e] = idx[e];
        }
        __syncthreads();
    }
    // rank of every row = sum over chunks of its lower-bound position (keys then row position);
    // the searches read the sorted chunks from LDS when the whole date fits
    const bool in_lds = n <= lds_rows;
    u64* LK = reinterpret_cast<u64*>(dyn);
    int32_t* LI = reinterpret_cast<int32_t*>(dyn + sizeof(u64) * (size_t)lds_rows);
    if (in_lds && nch > 1) {
        for (int e = tid; e < n; e += kWT) {
            LK[e] = g.skey[base + e];
            LI[e] = g.sidx[base + e];
        }
        __syncthreads();
    }
    for (int e = tid; e < n; e += kWT) {
        const u64 k0 = okey(g.rows[base + e]);
        int less = 0, greater = 0;
        for (int c = 0; c < nch; ++c) {
            const int c0 = c * kChunk, len = min(kChunk, n - c0);
            const u64* K = in_lds ? (nch > 1 ? LK + c0 : key) : g.skey + base + c0;
            const int32_t* I = in_lds ? (nch > 1 ? LI + c0 : idx) : g.sidx + base + c0;
            // lb: first position with (key, idx) >= (k0, e)
            int lo = 0, hi = len;
            while (lo < hi) {
                int m = (lo + hi) >> 1;
                if (K[m] < k0 || (K[m] == k0 && I[m] < e)) lo = m + 1; else hi = m;
            }
            const int lb = lo;
            // first key >= k0, first key > k0
            lo = 0; hi = len;
            while (lo < hi) { int m = (lo + hi) >> 1; if (K[m] < k0) lo = m + 1; else hi = m; }
            const int lbk = lo;
            lo = 0; hi = len;
            while (lo < hi) { int m = (lo + hi) >> 1; if (K[m] <= k0) lo = m + 1; else hi = m; }
            const int ubk = lo;
            less += lb;                              // key < k0, or equal and earlier
            greater += (len - ubk) + (lb - lbk);     // key > k0, or equal and earlier
        }
        g.rank_asc[base + e] = less + 1;
        g.rank_desc[base + e] = greater + 1;
    }
}

// ---- A3/A4 without a sort: the decile layer and the top-10 of every row --------------------
// xs_stats needs of the ranks only (a) each row's layer = min(int(rank/n*10)+1, 10) (KKT:328-330)
// and (b) the rows of descending rank <= 10 with that rank (KKT:359-369).  The layer is monotone
// in the rank, so with R_l = the largest rank of layer <= l, layer(e) = 1 + #{l < 10 : (key_e, e)
// > the R_l-th smallest (key, position)}: nine order statistics, found by one radix select that
// narrows all nine prefixes in the same passes over register-resident keys, exact ties resolved
// by position.  The top 10 (key descending, position ascending) by the same select.  Outputs in
// xs_rank's convention for xs_stats: rank_asc = the first rank of the row's layer (xs_stats
// recomputes the same layer from it), rank_desc = the true rank of a top-10 row, n + 1 else.
constexpr int kLT = 512;                  // threads
constexpr int kLR = 24;                   // register keys per thread: n <= 12288
constexpr int kNTg = 10;                  // targets: 9 decile bounds + the 10th largest

struct LayerSmem {
    int hist[kNTg][256];
    u64 prefix[kNTg];
    int need[kNTg];
    int eqtot[kNTg];
    int rneed[kNTg];                      // target rank (1-based), 0 = no row
    int eqidx[kNTg];                      // the position of the target row
    int ntop;
    u64 topk[kTopK];
    int topi[kTopK];
};

__device__ __forceinline__ int layer_of(int r, int n) {
    int l = (int)((double)r / (double)n * kLayers) + 1;
    return l > kLayers ? kLayers : l;
}

__global__ __launch_bounds__(kLT) void xs_layers_kernel(RankArgs g) {
    AFM_TAIL_PRIO_SET();
    __shared__ LayerSmem sh;
    const int tid = threadIdx.x, lane = tid & 63;
    const int64_t t = blockIdx.x;
    const int n = g.nrows[t];
    const int64_t base = t * g.lda;
    if (n <= 0) return;
    // keys: ascending order key; the top-10 target runs on the complemented key (descending)
    u64 ks[kLR];
#pragma unroll
    for (int j = 0; j < kLR; ++j) {
        const int e = j * kLT + tid;
        ks[j] = e < n ? okey(g.rows[base + e]) : 0ull;
    }
    if (tid < kNTg) {
        int r;
        if (tid < kNTg - 1) {             // R_l: the largest rank with layer <= l (l = tid + 1)
            int lo = 0, hi = n;           // f(lo) <= l (f(0) := 0), f(hi + 1) > l or hi = n
            while (lo < hi) {
                const int m = (lo + hi + 1) >> 1;
                if (layer_of(m, n) <= tid + 1) lo = m; else hi = m - 1;
            }
            r = lo;
        } else {
            r = n >= kTopK ? kTopK : n;   // the 10th largest (or the n-th)
        }
        sh.rneed[tid] = r;
        sh.need[tid] = r;
        sh.prefix[tid] = 0ull;
        sh.eqidx[tid] = 0;
    }
    __syncthreads();
    u64 pmask = 0ull;
    for (int shift = 56; shift >= 0; shift -= 8) {
        for (int e = tid; e < kNTg * 256; e += kLT) (&sh.hist[0][0])[e] = 0;
        __syncthreads();
        if (shift == 56) {
            // every target's prefix is empty: one histogram of the top digit, copied to the
            // ascending targets and mirrored for the complemented one
#pragma unroll
            for (int j = 0; j < kLR; ++j)
                if (j * kLT + tid < n) atomicAdd(&sh.hist[0][ks[j] >> 56], 1);
            __syncthreads();
            if (tid < 256) {
                const int h = sh.hist[0][tid];
#pragma unroll
                for (int q = 1; q < kNTg - 1; ++q) sh.hist[q][tid] = h;
                sh.hist[kNTg - 1][255 - tid] = h;
            }
        } else {
            u64 pf[kNTg];
            bool act[kNTg];
#pragma unroll
            for (int q = 0; q < kNTg; ++q) {
                pf[q] = sh.prefix[q];
                act[q] = sh.need[q] > 0;
            }
#pragma unroll
            for (int j = 0; j < kLR; ++j) {
                if (j * kLT + tid < n) {
#pragma unroll
                    for (int q = 0; q < kNTg; ++q) {
                        const u64 kk = q < kNTg - 1 ? ks[j] : ~ks[j];
                        if (act[q] && (kk & pmask) == pf[q])
                            atomicAdd(&sh.hist[q][(kk >> shift) & 255], 1);
                    }
                }
            }
        }
        __syncthreads();
        // digit pick, target q on wave q % 4: the smallest digit d with cumulative count >= need
        for (int q = tid >> 6; q < kNTg; q += kLT / 64) {
            const int nd = sh.need[q];
            if (nd > 0) {
                const int h0 = sh.hist[q][4 * lane], h1 = sh.hist[q][4 * lane + 1],
                          h2 = sh.hist[q][4 * lane + 2], h3 = sh.hist[q][4 * lane + 3];
                const int s4 = h0 + h1 + h2 + h3;
                int P = s4;                                // inclusive prefix over lanes
                for (int o = 1; o < 64; o <<= 1) {
                    const int v = __shfl_up(P, o, 64);
                    if (lane >= o) P += v;
                }
                const u64 m = __ballot(P >= nd);
                const int L = __builtin_ctzll(m);
                if (lane == L) {
                    int acc = P - s4, d = 4 * L, hd = h0;
                    if (acc + h0 >= nd) { d = 4 * L; hd = h0; }
                    else if (acc + h0 + h1 >= nd) { d = 4 * L + 1; hd = h1; acc += h0; }
                    else if (acc + h0 + h1 + h2 >= nd) { d = 4 * L + 2; hd = h2; acc += h0 + h1; }
                    else { d = 4 * L + 3; hd = h3; acc += h0 + h1 + h2; }
                    sh.prefix[q] |= (u64)d << shift;
                    sh.need[q] = nd - acc;
                    sh.eqtot[q] = hd;
                }
            }
        }
        pmask |= 255ull << shift;
        __syncthreads();
    }
    // ties at each target's key: the need-th smallest position among them, by the same select
    // over the positions (14 bits: two passes of 7)
    {
        int epfx[kNTg];
#pragma unroll
        for (int q = 0; q < kNTg; ++q) epfx[q] = 0;
        int emask = 0;
        for (int shift = 7; shift >= 0; shift -= 7) {
            for (int e = tid; e < kNTg * 256; e += kLT) (&sh.hist[0][0])[e] = 0;
            u64 pf[kNTg];
            bool act[kNTg];
#pragma unroll
            for (int q = 0; q < kNTg; ++q) {
                pf[q] = sh.prefix[q];
                act[q] = sh.need[q] > 0;
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kLR; ++j) {
                const int e = j * kLT + tid;
                if (e < n) {
#pragma unroll
                    for (int q = 0; q < kNTg; ++q) {
                        const u64 kk = q < kNTg - 1 ? ks[j] : ~ks[j];
                        if (act[q] && kk == pf[q] && (e & emask) == epfx[q])
                            atomicAdd(&sh.hist[q][(e >> shift) & 127], 1);
                    }
                }
            }
            __syncthreads();
            for (int q = tid >> 6; q < kNTg; q += kLT / 64) {
                const int nd = sh.need[q];
                if (nd > 0) {
                    const int h0 = sh.hist[q][2 * lane], h1 = sh.hist[q][2 * lane + 1];
                    const int s2 = h0 + h1;
                    int P = s2;
                    for (int o = 1; o < 64; o <<= 1) {
                        const int v = __shfl_up(P, o, 64);
                        if (lane >= o) P += v;
                    }
                    const u64 m = __ballot(P >= nd);
                    const int L = __builtin_ctzll(m);
                    if (lane == L) {
                        const int acc = P - s2;
                        const int d = acc + h0 >= nd ? 2 * L : 2 * L + 1;
                        sh.eqidx[q] = (shift == 7 ? 0 : sh.eqidx[q]) | (d << shift);
                        sh.need[q] = nd - (acc + h0 >= nd ? acc : acc + h0);
                    }
                }
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < kNTg; ++q) epfx[q] = sh.need[q] > 0 ? sh.eqidx[q] : 0;
            emask |= 127 << shift;
            __syncthreads();
        }
    }
    // layers; the top-10 rows (keys >= the 10th largest in (key desc, position asc) order)
    u64 kq[kNTg];
    int iq[kNTg];
    bool has[kNTg];
#pragma unroll
    for (int q = 0; q < kNTg; ++q) {
        kq[q] = sh.prefix[q];
        iq[q] = sh.eqidx[q];
        has[q] = sh.rneed[q] > 0;
    }
    int r0[kLayers];                                  // first rank of each layer
    r0[0] = 1;
#pragma unroll
    for (int l = 1; l < kLayers; ++l) r0[l] = sh.rneed[l - 1] + 1;
    if (tid == 0) sh.ntop = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kLR; ++j) {
        const int e = j * kLT + tid;
        if (e < n) {
            int l = 0;
#pragma unroll
            for (int q = 0; q < kNTg - 1; ++q)
                l += !has[q] || ks[j] > kq[q] || (ks[j] == kq[q] && e > iq[q]) ? 1 : 0;
            int rl = r0[0];
#pragma unroll
            for (int q = 1; q < kLayers; ++q) rl = l == q ? r0[q] : rl;
            g.rank_asc[base + e] = rl;
            const u64 kd = ~ks[j];                    // descending order key
            const int q = kNTg - 1;
            const bool top = kd < kq[q] || (kd == kq[q] && e <= iq[q]);
            g.rank_desc[base + e] = n + 1;
            if (top) {
                const int s = atomicAdd(&sh.ntop, 1);
                sh.topk[s] = kd;
                sh.topi[s] = e;
            }
        }
    }
    __syncthreads();
    const int ntop = sh.ntop;
    if (tid < ntop) {                                 // rank among the top rows by counting
        const u64 mk = sh.topk[tid];
        const int mi = sh.topi[tid];
        int rk = 1;
        for (int f = 0; f < ntop; ++f)
            rk += sh.topk[f] < mk || (sh.topk[f] == mk && sh.topi[f] < mi);
        g.rank_desc[base + mi] = rk;
    }
}

// ---- A2-A4: per (date, return type) sequential statistics --------------------------------------
struct StatArgs {
    int64_t T, lda;
    const int32_t* dates;     // [nd] dates to evaluate
    int64_t nd;
    const double* rows;       // [4][T][lda]
    const int32_t* nrows;
    const int32_t* rank_asc;
    const int32_t* rank_desc;
    int mcols;                // pivot columns present (ranks 1..mcols)
    double* ic;               // [nd][3]
    double* layer_mean;       // [nd][3][10]
    int32_t* layer_cnt;       // [nd][10]
    double* port;             // [nd][3]
};

// One workgroup (2 waves) per date.  Rows are staged through LDS in chunks (all 128 threads:
// the 4 value columns, each row's decile layer from its rank, the top-10 pivot cells); then the
// sequential recurrences run in lanes, each over the rows in order -- the operations of the
// reference, only spread over lanes:
//   wave 0, lanes 0..2    nancorr Welford of (return_k, factor) (KKT:344-345)
//   wave 1, lanes 0..29   Kahan group mean of return_k over the rows of layer l (k = lane / 10,
//                         l = lane % 10; groupby(['date', 'layer']).mean(), KKT:331-332)
// and lanes 0..2 of wave 0 finish the factor-weighted top-10 sums (KKT:362-369).
constexpr int kStatRows = 512;

__global__ __launch_bounds__(128) void xs_stats_kernel(StatArgs g) {
    AFM_TAIL_PRIO_SET();
    __shared__ double sv[4][kStatRows];          // factor, return_1, return_2, return_5
    __shared__ int8_t slay[kStatRows];
    __shared__ double sinv[kStatRows];           // 1 / (row number): the Welford divisor when no
                                                 // row has been skipped (IEEE, as 1. / nobs)
    __shared__ double pv_f[kTopK], pv_r[3][kTopK];
    __shared__ int pv_has[kTopK];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t di = blockIdx.x;
    const int64_t t = g.dates[di];
    const int n = g.nrows[t];
    const int64_t plane = g.T * g.lda;
    const int64_t base = t * g.lda;
    if (tid < kTopK) { pv_has[tid] = 0; pv_f[tid] = qnan(); }
    if (tid < 3 * kTopK) pv_r[tid / kTopK][tid % kTopK] = qnan();
    // wave 0 lanes 0..2: Welford state; wave 1 lanes 0..29: Kahan state
    const int k0 = lane;                                   // wave 0: return type
    const int k1 = lane / kLayers, l1 = lane % kLayers;    // wave 1: (type, layer)
    double nobs = 0, mx = 0, my = 0, sxx = 0, syy = 0, sxy = 0;
    double lsum = 0, lcomp = 0;
    int lcnt = 0;
    for (int c0 = 0; c0 < n; c0 += kStatRows) {
        const int len = min(kStatRows, n - c0);
        // the chunk's loads, all issued before any LDS write (round 4: a row-by-row copy waited
        // one global-load latency per row of each thread, and the whole per-date kernel was that
        // wait: 0.55 ms per date with or without the sequential lanes)
        constexpr int kPer = kStatRows / 128;
        double lv[kPer][4];
        int lra[kPer], lrd[kPer];
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int e = tid + 128 * u;
            const int64_t o = base + c0 + (e < len ? e : 0);
            lv[u][0] = g.rows[o];
#pragma unroll
            for (int q = 0; q < 3; ++q) lv[u][1 + q] = g.rows[(1 + q) * plane + o];
            lra[u] = g.rank_asc[o];
            lrd[u] = g.rank_desc[o];
        }
        __syncthreads();                                   // the previous chunk is consumed
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int e = tid + 128 * u;
            if (e >= len) continue;
#pragma unroll
            for (int q = 0; q < 4; ++q) sv[q][e] = lv[u][q];
            sinv[e] = 1. / (double)(c0 + e + 1);
            const double pct = (double)lra[u] / (double)n;              // KKT:328-330
            int layer = (int)(pct * kLayers) + 1;
            if (layer > kLayers) layer = kLayers;
            slay[e] = (int8_t)(layer - 1);
            const int rd = lrd[u];
            if (rd <= kTopK) {
                pv_f[rd - 1] = lv[u][0];
#pragma unroll
                for (int q = 0; q < 3; ++q) pv_r[q][rd - 1] = lv[u][1 + q];
                pv_has[rd - 1] = 1;
            }
        }
        // one flag for the chunk: every staged value finite (the analyzer's rows always are)
        int fin = 1;
#pragma unroll
        for (int u = 0; u < kPer; ++u)
            if (tid + 128 * u < len)
                fin &= __builtin_isfinite(lv[u][0]) && __builtin_isfinite(lv[u][1]) &&
                       __builtin_isfinite(lv[u][2]) && __builtin_isfinite(lv[u][3]);
        const bool all_fin = __syncthreads_and(fin);
        if (wave == 0 && lane < 3) {
            const double* R = sv[1 + k0];
            if (all_fin && nobs == (double)c0) {
                // no row skipped so far: nobs == row number, 1 / nobs from the table, no branch.
                // Blocks of 8 rows whose LDS values were read during the previous block (the
                // recurrences' chain -- sub, mul, add per row -- never waits for LDS), the tail
                // row by row
                auto step = [&](double vy, double vx, double inv) {
                    const double dx = vx - mx, dy = vy - my;
                    mx += inv * dx;
                    my += inv * dy;
                    sxx += (vx - mx) * dx;
                    syy += (vy - my) * dy;
                    sxy += (vx - mx) * dy;
                };
                constexpr int kB = 8;
                const int nb = len / kB;
                double ny[kB], nx[kB], ni[kB];
                if (nb > 0) {
#pragma unroll
                    for (int u = 0; u < kB; ++u) { ny[u] = sv[0][u]; nx[u] = R[u]; ni[u] = sinv[u]; }
                }
                for (int b = 0; b < nb; ++b) {
                    double y[kB], x[kB], iv[kB];
#pragma unroll
                    for (int u = 0; u < kB; ++u) { y[u] = ny[u]; x[u] = nx[u]; iv[u] = ni[u]; }
                    const int e1 = (b + 1 < nb ? b + 1 : b) * kB;   // (the last block re-reads)
#pragma unroll
                    for (int u = 0; u < kB; ++u) {
                        ny[u] = sv[0][e1 + u]; nx[u] = R[e1 + u]; ni[u] = sinv[e1 + u];
                    }
#pragma unroll
                    for (int u = 0; u < kB; ++u) step(y[u], x[u], iv[u]);
                }
                for (int e = nb * kB; e < len; ++e) step(sv[0][e], R[e], sinv[e]);
                nobs += (double)len;
            } else {
                for (int e = 0; e < len; ++e) {
                    const double vy = sv[0][e], vx = R[e];
                    if (__builtin_isfinite(vx) && __builtin_isfinite(vy)) {
                        nobs += 1;
                        const double dx = vx - mx, dy = vy - my;
                        const double inv = nobs == (double)(c0 + e + 1) ? sinv[e] : 1. / nobs;
                        mx += inv * dx;
                        my += inv * dy;
                        sxx += (vx - mx) * dx;
                        syy += (vy - my) * dy;
                        sxy += (vx - mx) * dy;
                    }
                }
            }
        } else if (wave == 1) {
            // each lane (type k1, layer l1) walks only its layer's rows: per 64-row group, one
            // ballot per layer, then the set bits in row order
            const double* R = sv[1 + (k1 < 3 ? k1 : 0)];
            for (int g0 = 0; g0 < len; g0 += 64) {
                const int e = g0 + lane;
                const int myl = e < len ? slay[e] : -1;
                u64 mine = 0ull;
#pragma unroll
                for (int l = 0; l < kLayers; ++l) {
                    const u64 m = __ballot(myl == l);
                    if (l == l1) mine = m;
                }
                if (lane < 3 * kLayers) {
                    while (mine) {
                        const int b = __builtin_ctzll(mine);
                        mine &= mine - 1;
                        const double vx = R[g0 + b];
                        if (vx == vx) {
                            lcnt += 1;
                            const double y = vx - lcomp;
                            const double tt = lsum + y;
                            lcomp = tt - lsum - y;
                            if (lcomp != lcomp) lcomp = 0;
                            lsum = tt;
                        }
                    }
                }
            }
        }
    }
    __syncthreads();
    if (wave == 1 && lane < 3 * kLayers) {
        g.layer_mean[(di * 3 + k1) * kLayers + l1] = lcnt ? lsum / (double)lcnt : qnan();
        if (k1 == 0) g.layer_cnt[di * kLayers + l1] = lcnt;
    }
    if (wave == 0 && lane < 3) {
        const int k = k0;
        double r = qnan();
        if (nobs >= 1) {
            const double div = __builtin_sqrt(sxx * syy);
            if (div != 0) r = sxy / div;
        }
        g.ic[di * 3 + k] = r;
        // pivot columns in string order '1.0','10.0','2.0',...,'9.0' (or 1..m for m < 10)
        int order[kTopK];
        const int m = g.mcols;
        if (m >= 10) {
            order[0] = 1; order[1] = 10;
            for (int j = 2; j < 10; ++j) order[j] = j;
        } else {
            for (int j = 0; j < m; ++j) order[j] = j + 1;
        }
        double row[kTopK];
        for (int j = 0; j < m; ++j) {
            const double f = pv_has[order[j] - 1] ? pv_f[order[j] - 1] : qnan();
            row[j] = f == f ? f : 0.0;
        }
        const double wsum = leaf_sum(row, m);
        for (int j = 0; j < m; ++j) {
            const int q = order[j] - 1;
            double v = qnan();
            if (pv_has[q]) v = pv_r[k][q] * (pv_f[q] / wsum);
            row[j] = v == v ? v : 0.0;
        }
        g.port[di * 3 + k] = leaf_sum(row, m);
    }
}

// ---- series: cumulative layers / long-short / top-k, per-year IR -----------------------------
__device__ double seq_pairwise(const double* a, int64_t n) {   // numpy pairwise_sum, one thread
    if (n <= 128) return leaf_sum(a, (int)n);
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return seq_pairwise(a, n2) + seq_pairwise(a + n2, n - n2);
}
__device__ double seq_np_sum(const double* a, int64_t n) {      // np.add.reduce (block_np_sum)
    double r = 0.0;
    for (int64_t c0 = 0; c0 < n; c0 += kNpBuf) r = r + seq_pairwise(a + c0, n - c0 < kNpBuf ? n - c0 : kNpBuf);
    return r;
}

// One workgroup.  Every series is a sequential recurrence over the dates, so each runs in one
// lane; its inputs are read in batches of kSerB (all issued before the batch's dependent sums and
// stores), and the per-year IC samples of the IR sit in LDS when they fit (at most 366 dates a
// year): a lane that waited for each date's load in turn took ~0.5 ms for ~1,000 dates.
constexpr int kSerB = 16;
constexpr int kSerYearCap = 366;

template <bool LDS_IR>
__global__ __launch_bounds__(1024) void xs_series_kernel(int64_t nd, const double* layer_mean,
                                                         const double* port, const double* ic,
                                                         const int32_t* year, int nyears,
                                                         int year0, double* cum_layer, double* ls,
                                                         double* cum_port, double* ir,
                                                         double* scratch) {
    AFM_TAIL_PRIO_SET();
    extern __shared__ double ir_lds[];                     // [3 * nyears][kSerYearCap]
    const int tid = threadIdx.x;
    if (tid < 30) {                                        // (type, layer) cumsum, NaN-skipping
        const int k = tid / 10, l = tid % 10;
        double s = 0.0;
        for (int64_t i0 = 0; i0 < nd; i0 += kSerB) {
            double xb[kSerB];
#pragma unroll
            for (int j = 0; j < kSerB; ++j)
                xb[j] = i0 + j < nd ? layer_mean[((i0 + j) * 3 + k) * kLayers + l] : 0.0;
#pragma unroll
            for (int j = 0; j < kSerB; ++j) {
                if (i0 + j >= nd) break;
                const double x = xb[j];
                double* o = &cum_layer[((i0 + j) * 3 + k) * kLayers + l];
                if (x == x) {
                    s = s + x;
                    *o = s;
                } else {
                    *o = qnan();
                }
            }
        }
    } else if (tid < 33) {
        const int k = tid - 30;
        double s = 0.0;
        for (int64_t i0 = 0; i0 < nd; i0 += kSerB) {
            double xb[kSerB];
#pragma unroll
            for (int j = 0; j < kSerB; ++j) xb[j] = i0 + j < nd ? port[(i0 + j) * 3 + k] : 0.0;
#pragma unroll
            for (int j = 0; j < kSerB; ++j) {
                if (i0 + j >= nd) break;
                s = s + xb[j];
                cum_port[(i0 + j) * 3 + k] = s;
            }
        }
    }
    __syncthreads();
    if (tid < 15) {                                        // long-short: cum[10-l+1] - cum[l]
        const int k = tid / 5, l = tid % 5 + 1;
        for (int64_t i0 = 0; i0 < nd; i0 += kSerB) {
            double hb[kSerB], lb[kSerB];
#pragma unroll
            for (int j = 0; j < kSerB; ++j) {
                const int64_t i = i0 + j < nd ? i0 + j : nd - 1;
                hb[j] = cum_layer[(i * 3 + k) * kLayers + (kLayers - l)];
                lb[j] = cum_layer[(i * 3 + k) * kLayers + (l - 1)];
            }
#pragma unroll
            for (int j = 0; j < kSerB; ++j)
                if (i0 + j < nd) ls[((i0 + j) * 3 + k) * 5 + (l - 1)] = hb[j] - lb[j];
        }
    }
    if (tid >= 64 && tid < 64 + 3 * nyears) {              // IR per (year, type)
        const int q = tid - 64;
        const int y = q / 3, k = q % 3;
        double* buf = LDS_IR ? ir_lds + (int64_t)q * kSerYearCap : scratch + (int64_t)q * nd;
        int64_t n = 0;
        for (int64_t i0 = 0; i0 < nd; i0 += kSerB) {
            double xb[kSerB];
            int yb[kSerB];
#pragma unroll
            for (int j = 0; j < kSerB; ++j) {
                const int64_t i = i0 + j < nd ? i0 + j : nd - 1;
                xb[j] = ic[i * 3 + k];
                yb[j] = year[i];
            }
#pragma unroll
            for (int j = 0; j < kSerB; ++j)
                if (i0 + j < nd && yb[j] == year0 + y && xb[j] == xb[j]) buf[n++] = xb[j];
        }
        double res = qnan();
        if (n > 0) {
            const double mean = seq_np_sum(buf, n) / (double)n;
            double sd = qnan();
            if (n > 1) {
                const double avg = seq_np_sum(buf, n) / (double)n;
                for (int64_t i = 0; i < n; ++i) {
                    const double d = avg - buf[i];
                    buf[i] = d * d;
                }
                sd = __builtin_sqrt(seq_np_sum(buf, n) / ((double)n - 1.0));
            }
            res = mean / sd;
        }
        ir[y * 3 + k] = res;
    }
}

// ---- §8(f) rank 2: ingest / clean (merge_datasets, KKT:113-166) ---------------------------
// ffill of each value column per security over the union (date, id) rows in date order
// (KKT:145): one thread per (column, asset), walking the presence words.
__global__ __launch_bounds__(256) void ffill_kernel(int64_t K, int64_t T, int64_t lda,
                                                    double* planes, const uint64_t* bits) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= K * lda) return;
    const int64_t k = i / lda, a = i - k * lda;
    double* col = planes + k * T * lda + a;
    double last = qnan();
    const int64_t nch = (T + 63) / 64;
    for (int64_t ch = 0; ch < nch; ++ch) {
        u64 w = bits[ch * lda + a];
        while (w) {
            const int64_t t = ch * 64 + __builtin_ctzll(w);
            w &= w - 1;
            double* cell = col + t * lda;
            const double v = *cell;
            if (v == v) last = v;
            else if (last == last) *cell = last;
        }
    }
}

// per-date mean fill (KKT:147): for date t and column k, the NaN cells of the date's rows take
// the column's mean over those rows -- pandas nanmean: numpy pairwise sum of the rows in
// security order with NaN -> 0, divided by the non-NaN count (NaN when none).
__global__ __launch_bounds__(kT) void date_mean_fill_kernel(int64_t K, int64_t T, int64_t A,
                                                            int64_t lda, double* planes,
                                                            const uint64_t* bits,
                                                            double* scratch) {
    __shared__ PwShared pw;
    __shared__ int sbuf[kT];
    __shared__ int cbuf[kT];
    const int tid = threadIdx.x;
    const int64_t t = blockIdx.x, k = blockIdx.y;
    double* row = planes + (k * T + t) * lda;
    double* scr = scratch + (k * T + t) * lda;
    int n = 0, cnt = 0;
    for (int64_t base = 0; base < A; base += kT) {
        const int64_t a = base + tid;
        int ok = 0;
        double v = 0.0;
        if (a < A && bit_at(bits, lda, t, a)) {
            ok = 1;
            v = row[a];
        }
        int ex;
        const int tot = block_scan(ok, sbuf, &ex);
        if (ok) scr[n + ex] = v == v ? v : 0.0;
        n += tot;
        int cex;
        cnt += block_scan(ok && v == v, cbuf, &cex);
    }
    __syncthreads();
    if (n == 0 || cnt == n) return;                 // no row / nothing to fill (uniform)
    const double mean = cnt > 0 ? block_np_sum(pw, scr, n) / (double)cnt : qnan();
    for (int64_t a = tid; a < A; a += kT)
        if (bit_at(bits, lda, t, a) && !(row[a] == row[a])) row[a] = mean;
}

// x - mean(x) per group of consecutive rows (Series.mean: numpy pairwise sum / count of the
// non-NaN values): excess_ret1d per date over the reference rows in file order (KKT:154-161).
__global__ __launch_bounds__(kT) void group_demean_kernel(const int64_t* offsets, const double* x,
                                                          double* out, double* scratch) {
    __shared__ PwShared pw;
    __shared__ int cbuf[kT];
    const int tid = threadIdx.x;
    const int64_t g = blockIdx.x;
    const int64_t o = offsets[g], n = offsets[g + 1] - o;
    int cnt = 0;
    for (int64_t base = 0; base < n; base += kT) {
        const int64_t i = base + tid;
        int ok = 0;
        if (i < n) {
            const double v = x[o + i];
            ok = v == v;
            scratch[o + i] = ok ? v : 0.0;
        }
        int ex;
        cnt += block_scan(ok, cbuf, &ex);
    }
    __syncthreads();
    const double mean = cnt > 0 ? block_np_sum(pw, scratch + o, n) / (double)cnt : qnan();
    for (int64_t i = tid; i < n; i += kT) out[o + i] = x[o + i] - mean;
}

}  // namespace
}  // namespace afm

using namespace afm;

extern "C" int afm_fwd_returns_f64(afm_ctx* ctx, int64_t T, int64_t lda, const double* close,
                                   const uint64_t* price_bits, double* fr) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(T > 0 && lda > 0 && lda % 64 == 0, "bad shape");
    AFM_CHECK_ARG(close && price_bits && fr, "null buffer");
    dim3 grid((unsigned)(lda / 64), (unsigned)((T + 3) / 4));
    hipLaunchKernelGGL(fwd_returns_kernel, grid, dim3(256), 0, ctx->stream, T, lda, close,
                       price_bits, fr);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_xs_prepare_range_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda,
                                        int64_t t0, int64_t t1, const double* sig,
                                        const double* fr, double* scratch, double* rows,
                                        int32_t* rows_idx, int32_t* nrows) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(T > 0 && A > 0 && lda >= A && lda % 64 == 0 && A <= 64 * kMaxWords,
                  "bad shape (A <= 32768)");
    AFM_CHECK_ARG(0 <= t0 && t0 <= t1 && t1 <= T, "bad date range");
    AFM_CHECK_ARG(sig && fr && scratch && rows && rows_idx && nrows, "null buffer");
    if (t1 == t0) return AFM_OK;
    PrepArgs g{T, lda, A, sig, fr, scratch, rows, rows_idx, nrows, t0, nullptr, nullptr};
#ifdef AFM_PROBE                     // profiling build (make prof): phase timestamps
    const bool probe = getenv("AFM_AN_PROBE") != nullptr;
#else
    const bool probe = false;
#endif
    if (probe) AFM_HIP(hipMalloc((void**)&g.stamps, sizeof(int64_t) * T * 5));
    if (probe) AFM_HIP(hipMalloc((void**)&g.clk, sizeof(int64_t) * T * 2));
    hipLaunchKernelGGL(xs_prepare_kernel, dim3((unsigned)(t1 - t0)), dim3(kPT), 0, ctx->stream, g);
    AFM_HIP(hipGetLastError());
    if (probe) {                       // experiment: mean phase durations per date (100 MHz clock)
        std::vector<int64_t> h((size_t)T * 5);
        AFM_HIP(hipMemcpy(h.data(), g.stamps, sizeof(int64_t) * T * 5, hipMemcpyDeviceToHost));
        double acc[4] = {0, 0, 0, 0};
        int64_t s0 = h[t0 * 5], s1 = h[t0 * 5 + 4];
        for (int64_t t = t0; t < t1; ++t) {
            for (int j = 0; j < 4; ++j) acc[j] += (double)(h[t * 5 + j + 1] - h[t * 5 + j]);
            s0 = std::min(s0, h[t * 5]);
            s1 = std::max(s1, h[t * 5 + 4]);
        }
        const double f = 1.0 / (double)(t1 - t0) / 100.0;
        fprintf(stderr, "xs_prepare phases (us/date): masks %.1f prefix %.1f means %.1f rows %.1f; "
                "span %.1f us\n", acc[0] * f, acc[1] * f, acc[2] * f, acc[3] * f, (s1 - s0) / 100.0);
        AFM_HIP(hipFree(g.stamps));
        AFM_HIP(hipFree(g.clk));
    }
    return AFM_OK;
}

extern "C" int afm_xs_prepare_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda,
                                  const double* sig, const double* fr, double* scratch,
                                  double* rows, int32_t* rows_idx, int32_t* nrows) {
    return afm_xs_prepare_range_f64(ctx, T, A, lda, 0, T, sig, fr, scratch, rows, rows_idx,
                                    nrows);
}

extern "C" int afm_xs_rank_f64(afm_ctx* ctx, int64_t T, int64_t lda, const double* rows,
                               const int32_t* nrows, uint64_t* skey, int32_t* sidx,
                               int32_t* rank_asc, int32_t* rank_desc) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(T > 0 && lda % 64 == 0, "bad shape");
    AFM_CHECK_ARG(rows && nrows && skey && sidx && rank_asc && rank_desc, "null buffer");
    RankArgs g{T, lda, rows, nrows, (u64*)skey, sidx, rank_asc, rank_desc};
    // phase-2 LDS: 12 B per row, up to 144 KB (a date with more rows searches in global memory)
    const size_t sort_bytes = (sizeof(u64) + sizeof(int32_t)) * kChunk;
    int lds_rows = (int)(lda < 12288 ? lda : 12288);
    const size_t lds = std::max(sort_bytes, (size_t)lds_rows * 12);
    AFM_HIP(afm_lds_opt_in(ctx, (const void*)xs_rank_kernel, 12288 * 12));
    hipLaunchKernelGGL(xs_rank_kernel, dim3((unsigned)T), dim3(kWT), lds, ctx->stream, g,
                       lds_rows);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_xs_layers_f64(afm_ctx* ctx, int64_t T, int64_t lda, const double* rows,
                                 const int32_t* nrows, uint64_t* skey, int32_t* sidx,
                                 int32_t* rank_asc, int32_t* rank_desc) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(T > 0 && lda % 64 == 0, "bad shape");
    AFM_CHECK_ARG(rows && nrows && skey && sidx && rank_asc && rank_desc, "null buffer");
    if (lda > (int64_t)kLR * kLT)                  // wider dates: the sorting kernel
        return afm_xs_rank_f64(ctx, T, lda, rows, nrows, skey, sidx, rank_asc, rank_desc);
    RankArgs g{T, lda, rows, nrows, (u64*)skey, sidx, rank_asc, rank_desc};
    hipLaunchKernelGGL(xs_layers_kernel, dim3((unsigned)T), dim3(kLT), 0, ctx->stream, g);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_xs_stats_f64(afm_ctx* ctx, int64_t T, int64_t lda, const int32_t* dates,
                                int64_t nd, const double* rows, const int32_t* nrows,
                                const int32_t* rank_asc, const int32_t* rank_desc, int mcols,
                                double* ic, double* layer_mean, int32_t* layer_cnt,
                                double* port) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(mcols >= 0 && mcols <= kTopK, "mcols must be in [0, 10]");
    AFM_CHECK_ARG(dates && rows && nrows && rank_asc && rank_desc && ic && layer_mean &&
                      layer_cnt && port, "null buffer");
    if (nd <= 0) return AFM_OK;
    StatArgs g{T, lda, dates, nd, rows, nrows, rank_asc, rank_desc, mcols, ic, layer_mean,
               layer_cnt, port};
    hipLaunchKernelGGL(xs_stats_kernel, dim3((unsigned)nd), dim3(128), 0, ctx->stream, g);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_xs_series_f64(afm_ctx* ctx, int64_t nd, const double* layer_mean,
                                 const double* port, const double* ic, const int32_t* year,
                                 int nyears, int year0, double* cum_layer, double* ls,
                                 double* cum_port, double* ir, double* scratch) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(nyears >= 0 && 64 + 3 * nyears <= 1024, "too many years (max 320)");
    AFM_CHECK_ARG(layer_mean && port && ic && year && cum_layer && ls && cum_port && ir &&
                      scratch, "null buffer");
    if (nd <= 0) return AFM_OK;
    // the per-year IC samples in LDS when they fit (at most kSerYearCap dates a year)
    const size_t lds = sizeof(double) * (size_t)(3 * nyears) * kSerYearCap;
    if (lds <= 150 * 1024) {
        AFM_HIP(afm_lds_opt_in(ctx, (const void*)xs_series_kernel<true>, 150 * 1024));
        hipLaunchKernelGGL(xs_series_kernel<true>, dim3(1), dim3(1024), lds, ctx->stream, nd,
                           layer_mean, port, ic, year, nyears, year0, cum_layer, ls, cum_port, ir,
                           scratch);
    } else {
        hipLaunchKernelGGL(xs_series_kernel<false>, dim3(1), dim3(1024), 0, ctx->stream, nd,
                           layer_mean, port, ic, year, nyears, year0, cum_layer, ls, cum_port, ir,
                           scratch);
    }
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_ffill_f64(afm_ctx* ctx, int64_t K, int64_t T, int64_t lda, double* planes,
                             const uint64_t* bits) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(K >= 0 && T >= 0 && lda % 64 == 0, "bad panel shape");
    AFM_CHECK_ARG(planes && bits, "null buffer");
    if (K == 0 || T == 0 || lda == 0) return AFM_OK;
    hipLaunchKernelGGL(ffill_kernel, dim3((unsigned)((K * lda + 255) / 256)), dim3(256), 0,
                       ctx->stream, K, T, lda, planes, bits);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_date_mean_fill_f64(afm_ctx* ctx, int64_t K, int64_t T, int64_t A, int64_t lda,
                                      double* planes, const uint64_t* bits, double* scratch) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(K >= 0 && T >= 0 && A >= 0 && A <= lda && lda % 64 == 0, "bad panel shape");
    AFM_CHECK_ARG(A <= 65536, "at most 65536 securities per date");
    AFM_CHECK_ARG(K <= 65535, "at most 65535 value columns");
    AFM_CHECK_ARG(planes && bits && scratch, "null buffer");
    if (K == 0 || T == 0 || A == 0) return AFM_OK;
    hipLaunchKernelGGL(date_mean_fill_kernel, dim3((unsigned)T, (unsigned)K), dim3(kT), 0,
                       ctx->stream, K, T, A, lda, planes, bits, scratch);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_group_demean_f64(afm_ctx* ctx, int64_t ngroups, const int64_t* offsets,
                                    int64_t max_group, const double* x, double* out,
                                    double* scratch) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(ngroups >= 0 && max_group <= 65536, "at most 65536 rows per group");
    AFM_CHECK_ARG(offsets && x && out && scratch, "null buffer");
    if (ngroups == 0) return AFM_OK;
    hipLaunchKernelGGL(group_demean_kernel, dim3((unsigned)ngroups), dim3(kT), 0, ctx->stream,
                       offsets, x, out, scratch);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

// Cross-sectional regression: per-segment shifted Gram matrices on fp64
// MFMA, batched scaled-Cholesky OLS solves, the pooled (train+valid) OLS as an exact Chan
// combination of the per-segment moments, Fama-MacBeth statistics and predictions.
//
// A "segment" is the set of rows reduced into one Gram: one DATE of a calendar-grid panel
// (rows = the assets present that day, read straight from the factor planes), or one block of
// rows of a long design matrix (the LinearRegression drop-in, KKT:582-590).
//
// Gram kernel (one workgroup = 4 waves per segment, two workgroups per CU):
//   Z = [1, x_1 .. x_p, y] over the segment's usable rows (mask bit set and every value finite),
//   shifted by the first usable row s (Z - s keeps the moments well conditioned; column 0 is
//   not shifted), G' = sum_rows (z - s)(z - s)^T.  Rows are staged 64 at a time through an LDS
//   tile [feature][row] (row stride 66 doubles -> conflict-free fragment reads); the regressor
//   block X'X goes to v_mfma_f64_16x16x4_f64 over the NT(NT+1)/2 upper-triangle 16x16 tile pairs
//   (NT = ceil(p/16): p = 96 needs 21 pairs, not the 28 a padded [1, x, y] block would), while the
//   border (sums of x and y, x'y, y'y, row count) is accumulated on the VALU from the same
//   fragments.  Waves: 2 pair groups x 2 row halves; partial sums are combined in a fixed order,
//   so results are deterministic.  The shift is found in the first block holding a usable row;
//   later blocks subtract it while staging.
// Two passes (MI355X: f64 MFMA and VALU share the SIMD's f64 pipe -- tools/mfma_probe: a partner
// wave's VALU instruction issues only between MFMAs -- so every producer VALU instruction costs
// MFMA-pipe time): the FAST pass stages rows without the
// per-row finiteness check; any masked-in non-finite value makes its column's diagonal entry
// non-finite (d*d never returns to finite), so the REDO pass re-runs exactly those segments with
// the checked staging (rows with a non-finite value excluded).  On segments with no such row
// both stagings perform the same operations: results are identical to a checked-only run.
// The FAST pass also drops the per-block barrier: an S-slot LDS ring with ready / freed counters
// lets the producers run up to S blocks ahead (S = 3 at p = 96).
// Algorithmic work per segment: rows * (p+2)(p+3) flops over 8(p+1) B per row.
#include "afm_internal.h"

#include <cstdlib>

#pragma clang fp contract(off)

namespace afm {
namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
#ifdef AFM_FP_PROFILE
// profiling build only: per (workgroup, wave) [total cycles, cycles waiting at barriers]
__device__ long long g_gram_cycles[1 << 16];
#define GPROF_BAR(acc) { const long long _t = __builtin_readcyclecounter(); lds_barrier(); acc += __builtin_readcyclecounter() - _t; }
#else
#define GPROF_BAR(acc) lds_barrier();
#endif
typedef unsigned long long u64;

constexpr int kMaxTiles = 7;          // p + 2 <= 112
constexpr int kMaxF = kMaxTiles * 16;
constexpr int kRS = 66;               // LDS tile row stride (doubles)
constexpr int kRows = 64;             // rows staged per tile
constexpr int kThreads = 256;
#ifndef AFM_GRAM_PRIO
#define AFM_GRAM_PRIO 1
#endif

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

// upper-triangle tile pairs in J-major order: q -> (I, J), I <= J
template <int NT>
struct PairTab {
    static constexpr int NP = NT * (NT + 1) / 2;
    int I[NP], J[NP];
    constexpr PairTab() : I(), J() {
        int q = 0;
        for (int j = 0; j < NT; ++j)
            for (int i = 0; i <= j; ++i) { I[q] = i; J[q] = j; ++q; }
    }
};

// pairs [Q0, Q1) of the table (group 0: the first half, group 1: the rest -- it touches every
// tile, so it also owns the border sums)
template <int NT, int GRP>
struct Group {
    static constexpr int NP = NT * (NT + 1) / 2;
    static constexpr int Q0 = GRP == 0 ? 0 : NP / 2;
    static constexpr int Q1 = GRP == 0 ? NP / 2 : NP;
    static constexpr int NQ = Q1 - Q0;
    static constexpr int NQA = NQ > 0 ? NQ : 1;
    static constexpr int TMAX = GRP == 0 ? (NQ > 0 ? PairTab<NT>().J[Q1 - 1] + 1 : 0) : NT;
};

template <int NT, int S = 2>
struct GramSmem {
    static constexpr int NF = NT * 16;
    static constexpr int NP = NT * (NT + 1) / 2;
    static constexpr int TROWS = NF + 2;             // x rows (zero padded), y row NF, dump NF+1
    // the epilogue reuses the tiles for the second row half's partial sums
    static constexpr int RED = NP * 256 + (2 * NT + 3) * 64;
    static_assert(S * TROWS * kRS >= RED, "epilogue scratch must fit in the tiles");
    double tile[S][TROWS][kRS];                      // S-slot ring of 64-row blocks
    int ready[S];                                    // FAST: producer stagings of the slot so far
    int freed[S];                                    // FAST: consumer releases of the slot so far
    double shs[NF + 2];                              // shifts of the tile rows (dump row: 0)
    int rowbad[2][kRows];                            // == b: row of block b is masked in but non-finite
    int anybad[2];                                   // == b: block b has such a row
    int cnt[kRows];                                  // usable rows, per lane (producer 0)
    int64_t coff[NF + 4];                            // element offset of staged feature f
    int found;
    int srow;                                        // the shift row (first usable row)
};

// ring depth of the FAST kernel: as many 64-row slots as fit in 160 KB of LDS (at most 4)
template <int NT>
constexpr int fast_slots() {
    constexpr int slot = (NT * 16 + 2) * kRS * 8;
    constexpr int n = (160 * 1024 - 4096) / slot;
    return n > 4 ? 4 : (n < 2 ? 2 : n);
}

// border sums (x, x*y) of tiles [LO, HI): split between the pair groups so that their VALU work
// balances (group 1 also owns sum y, sum y*y)
template <int NT, int GRP>
struct Border {
    static constexpr int T0 = Group<NT, 0>::TMAX < NT / 2 ? Group<NT, 0>::TMAX : NT / 2;
    static constexpr int LO = GRP == 0 ? 0 : T0;
    static constexpr int HI = GRP == 0 ? T0 : NT;
};

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// barrier ordering LDS only (a __syncthreads() would also drain the producers' prefetch loads)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// One staged block for a consumer wave.  Rows the mask leaves out, and masked-in rows with a
// non-finite value (zeroed by the producers' fix-up step), are zero in the tile.
template <int NT, int GRP, int S>
__device__ __forceinline__ void gram_block(GramSmem<NT, S>& sm, const int buf, const int kh, const int fi, const int kk,
                                           d4 (&acc)[Group<NT, GRP>::NQA], double (&bs)[NT],
                                           double (&bc)[NT], double& sy, double& syy) {
    using G = Group<NT, GRP>;
    using B = Border<NT, GRP>;
    constexpr int NF = NT * 16;
    constexpr PairTab<NT> tab{};
    constexpr int KS = kRows / 8;                    // k-steps per block of this row half
    constexpr bool WY = GRP == 1 || B::HI > B::LO;
    // fragments of k-step it: rows (kh + 2 it) * 4 + kk; two register sets in ping-pong (no
    // copies: every VALU instruction here is issue time the MFMA pipe loses)
    auto ld = [&](double (&f)[NT], double& y, int it) {
        const int a = (kh + 2 * it) * 4 + kk;
#pragma unroll
        for (int t = 0; t < G::TMAX; ++t) f[t] = sm.tile[buf][t * 16 + fi][a];
        if (WY) y = sm.tile[buf][NF][a];
    };
    auto step = [&](const double (&f)[NT], const double y) {
#pragma unroll
        for (int t = B::LO; t < B::HI; ++t) {
            bs[t] = bs[t] + f[t];
            bc[t] = __builtin_fma(f[t], y, bc[t]);
        }
        if (GRP == 1) {
            sy = sy + y;
            syy = __builtin_fma(y, y, syy);
        }
#pragma unroll
        for (int q = 0; q < G::NQ; ++q)
            acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(f[tab.I[G::Q0 + q]], f[tab.J[G::Q0 + q]],
                                                          acc[q], 0, 0, 0);
    };
    static_assert(KS % 2 == 0, "ping-pong needs an even k-step count");
    double fa[NT], fb[NT], ya = 0.0, yb = 0.0;
    ld(fa, ya, 0);
#pragma unroll
    for (int it = 0; it < KS; it += 2) {
        ld(fb, yb, it + 1);
        step(fa, ya);
        if (it + 2 < KS) ld(fa, ya, it + 2);
        step(fb, yb);
    }
}

template <int NT, int GRP, int S>
__device__ void gram_epilogue(const GramArgs& g, GramSmem<NT, S>& sm, const int kh, const int lane,
                              d4 (&acc)[Group<NT, GRP>::NQA], double (&bs)[NT], double (&bc)[NT],
                              double& sy, double& syy);

// Consumer wave (MFMA): pair group GRP, row half kh = wave & 1.  Block b lives in tile[b & 1].
template <int NT, int GRP>
__device__ void gram_consume(const GramArgs& g, GramSmem<NT>& sm, const int wave, const int lane,
                             const int nb) {
    using G = Group<NT, GRP>;
    using B = Border<NT, GRP>;
    constexpr PairTab<NT> tab{};
    const int kh = wave & 1;
    const int p = g.p;
    d4 acc[G::NQA];
#pragma unroll
    for (int q = 0; q < G::NQA; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
    double bs[NT], bc[NT];          // border: per lane sum x, sum x*y of tiles [LO, HI)
#pragma unroll
    for (int t = 0; t < NT; ++t) { bs[t] = 0.0; bc[t] = 0.0; }
    double sy = 0.0, syy = 0.0;
    const int fi = lane & 15, kk = lane >> 4;
    lds_barrier();                                   // block 0 staged
    long long twait = 0;
    const long long tstart = __builtin_readcyclecounter();
    for (int b = 0; b < nb; ++b) {
        const int buf = b & 1;
        if (__builtin_amdgcn_readfirstlane(sm.anybad[buf]) == b) lds_barrier();   // fix-up step
#if !defined(AFM_GRAM_SKIP) || AFM_GRAM_SKIP != 1      // experiments: producers alone
        gram_block<NT, GRP, 2>(sm, buf, kh, fi, kk, acc, bs, bc, sy, syy);
#endif
        GPROF_BAR(twait);                            // tile[buf] free, block b+1 staged
    }
#ifdef AFM_FP_PROFILE
    if (lane == 0 && blockIdx.x < 4096) {
        g_gram_cycles[(blockIdx.x * 8 + wave) * 2] = __builtin_readcyclecounter() - tstart;
        g_gram_cycles[(blockIdx.x * 8 + wave) * 2 + 1] = twait;
    }
#else
    (void)tstart;
    (void)twait;
#endif
    gram_epilogue<NT, GRP, 2>(g, sm, kh, lane, acc, bs, bc, sy, syy);
}

// Row half 1 parks its partials in the (now idle) tiles, row half 0 adds them (fixed order) and
// writes the segment's Gram.  Entered right after a barrier that every wave executes.
template <int NT, int GRP, int S>
__device__ void gram_epilogue(const GramArgs& g, GramSmem<NT, S>& sm, const int kh, const int lane,
                              d4 (&acc)[Group<NT, GRP>::NQA], double (&bs)[NT], double (&bc)[NT],
                              double& sy, double& syy) {
    using G = Group<NT, GRP>;
    using B = Border<NT, GRP>;
    constexpr PairTab<NT> tab{};
    const int p = g.p;
    const int p2 = p + 2;
    double* out = g.gram + (int64_t)blockIdx.x * p2 * p2;
    double* red = &sm.tile[0][0][0] + (GRP == 0 ? 0 : Group<NT, 0>::NQ * 256);
    double* rb = &sm.tile[0][0][0] + GramSmem<NT, S>::NP * 256;    // border partials
    if (kh == 1) {
#pragma unroll
        for (int q = 0; q < G::NQ; ++q)
#pragma unroll
            for (int r = 0; r < 4; ++r) red[(q * 4 + r) * 64 + lane] = acc[q][r];
#pragma unroll
        for (int t = B::LO; t < B::HI; ++t) {
            rb[t * 64 + lane] = bs[t];
            rb[(NT + t) * 64 + lane] = bc[t];
        }
        if (GRP == 1) {
            rb[(2 * NT) * 64 + lane] = sy;
            rb[(2 * NT + 1) * 64 + lane] = syy;
        }
    }
    lds_barrier();
    if (kh == 0) {
#pragma unroll
        for (int q = 0; q < G::NQ; ++q) {
            const int I = tab.I[G::Q0 + q], J = tab.J[G::Q0 + q];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double v = acc[q][r] + red[(q * 4 + r) * 64 + lane];
                const int row = I * 16 + (lane >> 4) + 4 * r;   // f64 MFMA C/D layout
                const int col = J * 16 + (lane & 15);
                if (row < p && col < p) {
                    out[(1 + row) * p2 + 1 + col] = v;
                    out[(1 + col) * p2 + 1 + row] = v;
                }
            }
        }
#pragma unroll
        for (int t = B::LO; t < B::HI; ++t) {
            rb[t * 64 + lane] = bs[t] + rb[t * 64 + lane];
            rb[(NT + t) * 64 + lane] = bc[t] + rb[(NT + t) * 64 + lane];
        }
        if (GRP == 1) {
            rb[(2 * NT) * 64 + lane] = sy + rb[(2 * NT) * 64 + lane];
            rb[(2 * NT + 1) * 64 + lane] = syy + rb[(2 * NT + 1) * 64 + lane];
        }
        lds_fence();
        // lane group kk holds rows == kk (mod 4): sum the 4 groups in order
        const int fend = p < B::HI * 16 ? p : B::HI * 16;
        for (int f = B::LO * 16 + lane; f < fend; f += 64) {
            const int t = f >> 4, c = f & 15;
            double s = 0.0, x = 0.0;
            for (int k4 = 0; k4 < 4; ++k4) {
                s = s + rb[t * 64 + k4 * 16 + c];
                x = x + rb[(NT + t) * 64 + k4 * 16 + c];
            }
            out[1 + f] = s;
            out[(1 + f) * p2] = s;
            out[(1 + f) * p2 + p + 1] = x;
            out[(p + 1) * p2 + 1 + f] = x;
        }
        if (GRP == 1 && lane == 0) {
            double s = 0.0, q = 0.0;
            for (int k4 = 0; k4 < 4; ++k4) {
                s = s + rb[(2 * NT) * 64 + k4 * 16];
                q = q + rb[(2 * NT + 1) * 64 + k4 * 16];
            }
            int n = 0;
            for (int a = 0; a < kRows; ++a) n += sm.cnt[a];
            out[0] = (double)n;
            out[p + 1] = s;
            out[(p + 1) * p2] = s;
            out[(p + 1) * p2 + p + 1] = q;
        }
    }
}

// Producer wave pw (0..3): features pw + 4 j of every block, global -> registers two blocks
// ahead -> tile[b & 1] minus the shift.  A row the mask leaves out is loaded from the SHIFT row
// instead, so it stages as exact zeros with no per-element select; a masked-in row with a
// non-finite value is flagged (rowbad / anybad) through a NaN-propagating x*0 sum.  Only loads:
// its prefetches are never held behind stores.  With f64 MFMA, every VALU instruction of either
// wave of a SIMD is issue time the matrix pipe loses, so this loop is written for VALU count.
template <int NT, bool FAST>
__device__ void gram_produce(const GramArgs& g, GramSmem<NT>& sm, const int pw, const int lane,
                             const int nb, const int64_t rmax) {
    constexpr int NF = NT * 16;
    constexpr int KPER = (NF + 4) / 4;
    const int64_t seg = g.seg0 + blockIdx.x;
    const int p = g.p;
    // per-lane constants of this wave's features f = pw + 4 j: source column, shift, tile row
    // (source pointers and tile rows are wave-uniform: forced into SGPRs, the shifts stay VGPRs)
    const double* src[KPER];
    double shv[KPER];
    auto lrow_of = [&](int j) {
        const int f = pw + 4 * j;
        return f < p ? f : (f == p ? NF : NF + 1);
    };
#pragma unroll
    for (int j = 0; j < KPER; ++j) {
        const int64_t o = sm.coff[pw + 4 * j];
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(uint64_t)o);
        const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((uint64_t)o >> 32));
        src[j] = g.base + (int64_t)(((uint64_t)hi << 32) | lo);
        shv[j] = sm.shs[lrow_of(j)];
    }
    const uint64_t* bits = g.bits ? g.bits + (seg >> 6) * g.seg_stride : nullptr;
    const int sb = (int)(seg & 63);
    const unsigned srow = (unsigned)sm.srow;
    // the mask word of a block is loaded two loads ahead of its data
    auto bits_load = [&](int b) -> uint64_t {
        if (!bits) return ~0ull;
        int64_t r = (int64_t)b * kRows + lane;
        r = r < rmax ? r : rmax;
        return bits[r];
    };
    // two blocks in flight per producer; register slots are compile-time (b & 1)
    double pre0[KPER], pre1[KPER];
    bool ok0 = false, ok1 = false;
    int cnt = 0;                                     // producer 0: usable rows of this lane
    bool okp = false;                                // producer 0: mask bit of the previous block
    auto load = [&](int b, double (&pre)[KPER], bool& ok, const uint64_t bw) {
#if defined(AFM_GRAM_SKIP) && AFM_GRAM_SKIP == 2       // experiments: consumers alone
        return;
#endif
        const int64_t r = (int64_t)b * kRows + lane;
        ok = r <= rmax && ((bw >> sb) & 1ull);
        const unsigned off = (ok ? (unsigned)r : srow) * 8u;
#pragma unroll
        for (int j = 0; j < KPER; ++j)
            pre[j] = *reinterpret_cast<const double*>(reinterpret_cast<const char*>(src[j]) + off);
    };
    auto stage = [&](int b, const double (&pre)[KPER], const bool ok) {
#if defined(AFM_GRAM_SKIP) && AFM_GRAM_SKIP == 2
        return;
#endif
        const int buf = b & 1;
        double* tb = &sm.tile[buf][0][0] + lane;
        if (FAST) {                                  // no check: anybad / rowbad stay -1
#pragma unroll
            for (int j = 0; j < KPER; ++j) tb[lrow_of(j) * kRS] = pre[j] - shv[j];
        } else {
            double chk = 0.0;
#pragma unroll
            for (int j = 0; j < KPER; ++j) {
                const double d = pre[j] - shv[j];
                chk = __builtin_fma(d, 0.0, chk);    // NaN iff some d is not finite
                tb[lrow_of(j) * kRS] = d;
            }
            const bool bad = !(chk == 0.0);
            if (bad) sm.rowbad[buf][lane] = b;                      // benign race: same value
            if (__ballot(bad) != 0ull && lane == 0) sm.anybad[buf] = b;
        }
        if (pw == 0) {
            // block b-1 is complete (a barrier separates the two stagings): count its rows
            if (okp && sm.rowbad[buf ^ 1][lane] != b - 1) ++cnt;
            okp = ok;
        }
    };
    // fix-up step, only for a block with a masked-in non-finite row (never on a pipeline mask,
    // which already excludes them): zero those rows before the consumers read the block
    auto fixup = [&](int b) {
        const int buf = b & 1;
        if (__builtin_amdgcn_readfirstlane(sm.anybad[buf]) != b) return;
        if (sm.rowbad[buf][lane] == b) {
            double* tb = &sm.tile[buf][0][0] + lane;
#pragma unroll
            for (int j = 0; j < KPER; ++j) tb[lrow_of(j) * kRS] = 0.0;
        }
        lds_barrier();
    };
    // the producers are the younger half: without priority they lose every VALU arbitration to
    // the MFMA waves of their SIMD (MI355X_MICROARCH.md, two waves per SIMD, item 4)
    if (AFM_GRAM_PRIO) __builtin_amdgcn_s_setprio(AFM_GRAM_PRIO);
    uint64_t bwA = bits_load(0), bwB = bits_load(1);
    load(0, pre0, ok0, bwA);
    bwA = bits_load(2);
    if (nb > 1) {
        load(1, pre1, ok1, bwB);
        bwB = bits_load(3);
    }
    stage(0, pre0, ok0);
    if (nb > 2) {
        load(2, pre0, ok0, bwA);
        bwA = bits_load(4);
    }
    lds_barrier();                                   // block 0 staged
    long long twait = 0;
    const long long tstart = __builtin_readcyclecounter();
    for (int b = 0; b < nb; b += 2) {
        // iteration b: stage b+1 (slot 1), refill slot 1 with b+3
        fixup(b);
        if (b + 1 < nb) {
            stage(b + 1, pre1, ok1);
            if (b + 3 < nb) {
                load(b + 3, pre1, ok1, bwB);
                bwB = bits_load(b + 5);
            }
        }
        GPROF_BAR(twait);
        if (b + 1 >= nb) break;
        // iteration b+1: stage b+2 (slot 0), refill slot 0 with b+4
        fixup(b + 1);
        if (b + 2 < nb) {
            stage(b + 2, pre0, ok0);
            if (b + 4 < nb) {
                load(b + 4, pre0, ok0, bwA);
                bwA = bits_load(b + 6);
            }
        }
        GPROF_BAR(twait);
    }
#ifdef AFM_FP_PROFILE
    if (lane == 0 && blockIdx.x < 4096) {
        g_gram_cycles[(blockIdx.x * 8 + 4 + pw) * 2] = __builtin_readcyclecounter() - tstart;
        g_gram_cycles[(blockIdx.x * 8 + 4 + pw) * 2 + 1] = twait;
    }
#else
    (void)tstart;
    (void)twait;
#endif
    if (pw == 0) {
        if (okp && sm.rowbad[(nb - 1) & 1][lane] != nb - 1) ++cnt;
        sm.cnt[lane] = cnt;
    }
    lds_barrier();                                   // the consumers' epilogue barrier
}

// ---- FAST pass: producers and consumers decoupled through an S-slot ring ------------------
// Lock-step barriers made every block cost max(producer, consumer) plus the skew of both (the
// producers' VALU issues only between the MFMAs of their SIMD partner, so their pace varies).
// Here block b lives in slot b % S; ready[slot] counts producer stagings, freed[slot] consumer
// releases (monotonic, one LDS atomic per wave and block).  Producers run up to S blocks ahead.
__device__ __forceinline__ int lds_load_relaxed(int* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void wait_count(int* p, int target) {
    while (__builtin_amdgcn_readfirstlane(lds_load_relaxed(p)) < target)
        __builtin_amdgcn_s_sleep(1);
}
// signal after every LDS access of this wave so far has completed
__device__ __forceinline__ void signal_count(int* p, int lane) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(p, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int NT, int GRP, int S>
__device__ void gram_consume_fast(const GramArgs& g, GramSmem<NT, S>& sm, const int wave,
                                  const int lane, const int nb) {
    using G = Group<NT, GRP>;
    const int kh = wave & 1;
    d4 acc[G::NQA];
#pragma unroll
    for (int q = 0; q < G::NQA; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
    double bs[NT], bc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) { bs[t] = 0.0; bc[t] = 0.0; }
    double sy = 0.0, syy = 0.0;
    const int fi = lane & 15, kk = lane >> 4;
    int slot = 0, gen = 1;
    for (int b = 0; b < nb; ++b) {
        wait_count(&sm.ready[slot], 4 * gen);
        gram_block<NT, GRP, S>(sm, slot, kh, fi, kk, acc, bs, bc, sy, syy);
        signal_count(&sm.freed[slot], lane);
        if (++slot == S) { slot = 0; ++gen; }
    }
    lds_barrier();                                   // every wave is done with the ring
    gram_epilogue<NT, GRP, S>(g, sm, kh, lane, acc, bs, bc, sy, syy);
}

template <int NT, int S>
__device__ void gram_produce_fast(const GramArgs& g, GramSmem<NT, S>& sm, const int pw,
                                  const int lane, const int nb, const int64_t rmax) {
    constexpr int NF = NT * 16;
    constexpr int KPER = (NF + 4) / 4;
    const int64_t seg = g.seg0 + blockIdx.x;
    const int p = g.p;
    const double* src[KPER];
    double shv[KPER];
    auto lrow_of = [&](int j) {
        const int f = pw + 4 * j;
        return f < p ? f : (f == p ? NF : NF + 1);
    };
#pragma unroll
    for (int j = 0; j < KPER; ++j) {
        const int64_t o = sm.coff[pw + 4 * j];
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(uint64_t)o);
        const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((uint64_t)o >> 32));
        src[j] = g.base + (int64_t)(((uint64_t)hi << 32) | lo);
        shv[j] = sm.shs[lrow_of(j)];
    }
    const uint64_t* bits = g.bits ? g.bits + (seg >> 6) * g.seg_stride : nullptr;
    const int sb = (int)(seg & 63);
    const unsigned srow = (unsigned)sm.srow;
    auto bits_load = [&](int b) -> uint64_t {
        if (!bits) return ~0ull;
        int64_t r = (int64_t)b * kRows + lane;
        r = r < rmax ? r : rmax;
        return bits[r];
    };
    double pre0[KPER], pre1[KPER];
    bool ok0 = false, ok1 = false;
    int cnt = 0;                                     // producer 0: usable rows of this lane
    auto load = [&](int b, double (&pre)[KPER], bool& ok, const uint64_t bw) {
        const int64_t r = (int64_t)b * kRows + lane;
        ok = r <= rmax && ((bw >> sb) & 1ull);
        const unsigned off = (ok ? (unsigned)r : srow) * 8u;
#pragma unroll
        for (int j = 0; j < KPER; ++j)
            pre[j] = *reinterpret_cast<const double*>(reinterpret_cast<const char*>(src[j]) + off);
    };
    int slot = 0, gen = 0;
    auto stage = [&](const double (&pre)[KPER], const bool ok) {
        wait_count(&sm.freed[slot], 4 * gen);        // the slot's previous block is consumed
        double* tb = &sm.tile[slot][0][0] + lane;
#pragma unroll
        for (int j = 0; j < KPER; ++j) tb[lrow_of(j) * kRS] = pre[j] - shv[j];
        if (pw == 0) cnt += ok ? 1 : 0;
        signal_count(&sm.ready[slot], lane);
        if (++slot == S) { slot = 0; ++gen; }
    };
    __builtin_amdgcn_s_setprio(AFM_GRAM_PRIO);
    uint64_t bwA = bits_load(0), bwB = bits_load(1);
    load(0, pre0, ok0, bwA);
    bwA = bits_load(2);
    if (nb > 1) {
        load(1, pre1, ok1, bwB);
        bwB = bits_load(3);
    }
    for (int b = 0; b < nb; b += 2) {
        stage(pre0, ok0);
        if (b + 2 < nb) {
            load(b + 2, pre0, ok0, bwA);
            bwA = bits_load(b + 4);
        }
        if (b + 1 >= nb) break;
        stage(pre1, ok1);
        if (b + 3 < nb) {
            load(b + 3, pre1, ok1, bwB);
            bwB = bits_load(b + 5);
        }
    }
    if (pw == 0) sm.cnt[lane] = cnt;
    lds_barrier();                                   // the consumers' ring-done barrier
    lds_barrier();                                   // the consumers' epilogue barrier
}

// One workgroup per segment: 4 consumer waves (2 pair groups x 2 row halves) + 4 producer
// waves; blocks of 64 rows double-buffered in LDS, one barrier per block.
// MODE 0: checked staging; 1: FAST pass; 2: REDO pass (checked, only segments whose FAST result
// has a non-finite diagonal entry -- the others exit at once).
template <int NT, int MODE>
__global__ __launch_bounds__(512, 1) void gram_kernel(GramArgs g) {
    constexpr int NF = NT * 16;
    constexpr int S = MODE == 1 ? fast_slots<NT>() : 2;
    constexpr int TROWS = GramSmem<NT, S>::TROWS;
    __shared__ GramSmem<NT, S> sm;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int p = g.p, p2 = p + 2;
    const int64_t seg = g.seg0 + blockIdx.x;
    const int64_t rowbase = seg * g.seg_stride;
    if (MODE == 2) {
        const double* G = g.gram + (int64_t)blockIdx.x * p2 * p2;
        bool bad = false;
        for (int f = 1 + tid; f < p2; f += 512) bad = bad || !__builtin_isfinite(G[f * p2 + f]);
        if (!__syncthreads_or(bad)) return;
    }
    for (int i = tid; i < S * TROWS * kRS; i += 512) (&sm.tile[0][0][0])[i] = 0.0;
    if (tid < S) { sm.ready[tid] = 0; sm.freed[tid] = 0; }
    for (int i = tid; i < NF + 4; i += 512) {
        if (i <= NF + 1) sm.shs[i] = 0.0;
        const int c = i < p ? g.cols[i] : g.ycol;
        sm.coff[i] = (int64_t)c * g.col_stride + rowbase;
    }
    if (tid < 2 * kRows) sm.rowbad[tid >> 6][tid & 63] = -1;
    if (tid < 2) sm.anybad[tid] = -1;
    if (tid == 0) sm.found = 0;
    int64_t rmax = g.seg_rows - 1;                   // last row of the segment (row_limit too)
    if (g.row_limit >= 0 && g.row_limit - 1 - rowbase < rmax) rmax = g.row_limit - 1 - rowbase;
    __syncthreads();
    // ---- the shift: first usable row (mask bit set, every staged column finite) ----
    if (wave == 0 && rmax >= 0) {
        int64_t srow = -1;
        for (int64_t r0 = 0; r0 <= rmax && srow < 0; r0 += kRows) {
            const int64_t r = r0 + lane;
            bool cand = r <= rmax;
            if (cand && g.bits) cand = (g.bits[(seg >> 6) * g.seg_stride + r] >> (seg & 63)) & 1ull;
            if (cand) cand = __builtin_isfinite(g.base[sm.coff[p] + r]);
            u64 m = __ballot(cand);
            while (m != 0ull) {
                const int64_t row = r0 + __builtin_ctzll(m);
                bool bad = false;
                for (int f = lane; f < p; f += 64) bad = bad || !__builtin_isfinite(g.base[sm.coff[f] + row]);
                if (__ballot(bad) == 0ull) { srow = row; break; }
                m &= m - 1;
            }
        }
        if (srow >= 0) {
            for (int f = lane; f < p; f += 64) sm.shs[f] = g.base[sm.coff[f] + srow];
            if (lane == 0) {
                sm.shs[NF] = g.base[sm.coff[p] + srow];
                sm.found = 1;
                sm.srow = (int)srow;
            }
        }
    }
    __syncthreads();
    if (!sm.found) {                                 // no usable row: n = 0
        double* out = g.gram + (int64_t)blockIdx.x * p2 * p2;
        for (int e = tid; e < p2 * p2; e += 512) out[e] = 0.0;
        if (tid < p2) g.shift[(int64_t)blockIdx.x * p2 + tid] = 0.0;
        return;
    }
    const int nb = (int)((rmax + kRows) / kRows);
    if constexpr (MODE == 1) {
        if (wave < 2) gram_consume_fast<NT, 0, S>(g, sm, wave, lane, nb);
        else if (wave < 4) gram_consume_fast<NT, 1, S>(g, sm, wave, lane, nb);
        else gram_produce_fast<NT, S>(g, sm, wave - 4, lane, nb, rmax);
    } else {
        if (wave < 2) gram_consume<NT, 0>(g, sm, wave, lane, nb);
        else if (wave < 4) gram_consume<NT, 1>(g, sm, wave, lane, nb);
        else gram_produce<NT, false>(g, sm, wave - 4, lane, nb, rmax);
    }
    if (tid < p2) {
        const double v = tid == 0 ? 0.0 : (tid <= p ? sm.shs[tid - 1] : sm.shs[NF]);
        g.shift[(int64_t)blockIdx.x * p2 + tid] = v;
    }
}

// ---- per-segment OLS from the shifted Gram -------------------------------------------------
// C = G'[1:,1:] - G'[0,1:] G'[0,1:]^T / n: centered moments of the AUGMENTED [x, y] (q = p + 1
// columns), x scaled to unit diagonal.  A right-looking Cholesky over the p x-columns also
// eliminates the y row, which leaves z = L^-1 r in it (forward substitution for free); a pivot
// below tol drops its regressor (beta = 0).  The factor is kept unscaled -- the update is
// M[i][j] -= M[i][k] M[j][k] / d_k -- so each column costs ONE barrier; back substitution
// beta_j = (M[y][j] - sum_{i>j} M[i][j] beta_i) / d_j runs in one wave.  beta = D b,
// intercept = ybar - xbar . beta.  One workgroup per segment, the lower triangle packed in LDS
// (row i at i(i+1)/2: 38 KB at p = 96, so four workgroups share a CU where the square layout's
// 76 KB allowed two; every access is on or below the diagonal).
struct SolveArgs {
    const double* gram;      // [nseg][pg + 2][pg + 2]
    const double* shift;     // [nseg][pg + 2]
    int p;
    double tol;
    const int32_t* sel;      // optional [p]: regressor i is Gram feature sel[i] (0-based); y = pg
    int pg;                  // features of the Gram (p when sel is null)
    double* beta;            // [nseg][p+1]: intercept, beta_1..p
    double* nobs;            // [nseg]
    int32_t* rank;           // [nseg]
};

constexpr int kMaxP = kMaxF - 2;

__global__ __launch_bounds__(kThreads) void ols_solve_kernel(SolveArgs s) {
    AFM_TAIL_PRIO_SET();
    extern __shared__ __attribute__((aligned(16))) double M[];    // packed lower triangle
    __shared__ double dsc[kMaxP + 1];
    __shared__ double dk[kMaxP];
    __shared__ double mean[kMaxP + 2];
    __shared__ double bvec[kMaxP];
    __shared__ int drop[kMaxP];
    __shared__ int gx[kMaxP + 2];                    // Gram index of augmented column r (0: ones)
    const int tid = threadIdx.x;
    const int p = s.p, q = p + 1;
    const int p2 = s.pg + 2;                         // Gram dimension
    auto row = [](int i) { return i * (i + 1) / 2; };      // offset of row i
    const double* G = s.gram + (int64_t)blockIdx.x * p2 * p2;
    const double* sf = s.shift + (int64_t)blockIdx.x * p2;
    for (int r = tid; r <= q; r += kThreads)
        gx[r] = r == 0 ? 0 : (r == q ? s.pg + 1 : (s.sel ? 1 + s.sel[r - 1] : r));
    __syncthreads();
    const double n = G[0];
    double* beta = s.beta + (int64_t)blockIdx.x * (p + 1);
    if (tid == 0) s.nobs[blockIdx.x] = n;
    if (!(n > (double)p)) {                          // under-determined segment
        for (int j = tid; j <= p; j += kThreads) beta[j] = __builtin_nan("");
        if (tid == 0) s.rank[blockIdx.x] = 0;
        return;
    }
    for (int j = tid; j <= q; j += kThreads) mean[j] = (j == 0) ? 1.0 : G[gx[j]] / n;   // shifted
    for (int r = tid; r < q; r += kThreads) {
        const int gr = gx[r + 1];
        const double d = G[gr * p2 + gr] - G[gr] * G[gr] / n;
        dsc[r] = r < p ? (d > 0 ? 1.0 / __builtin_sqrt(d) : 0.0) : 1.0;
        if (r < p) drop[r] = !(d > 0);
    }
    __syncthreads();
    // lower triangle of D C D (packed rows)
    for (int r = tid >> 4; r < q; r += kThreads >> 4)
        for (int c = tid & 15; c <= r; c += 16) {
            const int gr = gx[r + 1], gc = gx[c + 1];
            const double v = G[gr * p2 + gc] - G[gr] * G[gc] / n;
            M[row(r) + c] = v * dsc[r] * dsc[c];
        }
    __syncthreads();
    // right-looking Cholesky of the x block, thresholded; the y row rides along
    const int ty = tid >> 4, tx = tid & 15;
    for (int k = 0; k < p; ++k) {
        const double d = M[row(k) + k];
        const bool dr = drop[k] || !(d > s.tol);     // uniform: every thread reads the same
        if (!dr) {
            const double inv = 1.0 / d;
            for (int i = k + 1 + ty; i < q; i += 16) {
                const int ri = row(i);
                const double mik = M[ri + k] * inv;
                for (int j = k + 1 + tx; j <= i; j += 16)
                    M[ri + j] = M[ri + j] - mik * M[row(j) + k];
            }
        }
        if (tid == 0) { drop[k] = dr ? 1 : 0; dk[k] = d; }
        __syncthreads();
    }
    if (tid < 64) {                                  // back substitution, one wave
        const int lane = tid;
        double t0 = lane < p ? M[row(p) + lane] : 0.0;
        double t1 = lane + 64 < p ? M[row(p) + lane + 64] : 0.0;
        for (int k = p - 1; k >= 0; --k) {
            const double tk = __shfl(k >= 64 ? t1 : t0, k & 63, 64);
            const double bk = drop[k] ? 0.0 : tk / dk[k];
            if (lane == 0) bvec[k] = bk;
            if (lane < k) t0 = t0 - M[row(k) + lane] * bk;
            if (lane + 64 < k) t1 = t1 - M[row(k) + lane + 64] * bk;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // bvec visible to the wave
        double part = 0.0;                           // intercept = ybar - sum xbar_j b_j
        int rk = 0;
        for (int j = lane; j < p; j += 64) {
            const double b = bvec[j] * dsc[j];
            beta[1 + j] = b;
            part = part + (sf[gx[1 + j]] + mean[1 + j]) * b;
            rk += drop[j] ? 0 : 1;
        }
        for (int o = 32; o > 0; o >>= 1) {
            part = part + __shfl_xor(part, o, 64);
            rk += __shfl_xor(rk, o, 64);
        }
        if (lane == 0) {
            beta[0] = (sf[gx[q]] + mean[q]) - part;
            s.rank[blockIdx.x] = rk;
        }
    }
}

// ---- exact (Chan) combination of per-segment shifted moments ----------------------------------
// Block b combines segments [b*per, min((b+1)*per, nseg)) in order and emits the union's moments
// in the same "shifted" representation (G'[0][0] = n, G'[0][j] = 0, G'[i][j] = centered sums,
// shift = mean), so a next level (or ols_solve_kernel) consumes it unchanged.  pool_tree below
// fixes the tree (16, 4, then 8 per level): the same for any split of the segments into
// 64-aligned shards (multi-GPU).

// The lower triangle is split over gridDim.y workgroups per date block (kPoolPer elements per
// thread each): every element's chain of merges is independent of the others, so the split only
// shortens each thread's per-segment work (one division per element) and leaves every result
// bit-identical.  The merge scalars (n, Chan factor, means) are recomputed by each workgroup of
// the split.  The next segment's entries are prefetched while the current one is merged (two
// barriers per segment).
constexpr int kPoolPer = 4;

__global__ __launch_bounds__(kThreads) void pool_kernel(const double* gram, const double* shift,
                                                        int p2, int64_t nseg, int64_t per,
                                                        double* out_gram, double* out_shift) {
    __shared__ double mu[kMaxF];
    __shared__ double dl[kMaxF];
    __shared__ double g0[kMaxF];
    __shared__ double ntot_s, fac_s;
    const int tid = threadIdx.x;
    const int q2 = p2 * p2;
    const int q = p2 - 1;                              // rows / cols 1..q of the lower triangle
    const int nel = q * (q + 1) / 2;
    const int64_t s0 = (int64_t)blockIdx.x * per;
    const int64_t s1 = s0 + per < nseg ? s0 + per : nseg;
    const int ebase = (int)blockIdx.y * kPoolPer * kThreads;
    // my elements: e = ebase + tid + k * kThreads -> (r, c), 1 <= c <= r <= q
    int ro[kPoolPer], co[kPoolPer];
#pragma unroll
    for (int k = 0; k < kPoolPer; ++k) {
        const int e = ebase + tid + k * kThreads;
        int r = (int)((__builtin_sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
        while ((r + 1) * (r + 2) / 2 <= e) ++r;
        while (r * (r + 1) / 2 > e) --r;
        ro[k] = e < nel ? r + 1 : 1;
        co[k] = e < nel ? e - r * (r + 1) / 2 + 1 : 1;
    }
    double acc[kPoolPer], cur[kPoolPer], nxt[kPoolPer];
#pragma unroll
    for (int k = 0; k < kPoolPer; ++k) acc[k] = 0.0;
    if (tid < p2) mu[tid] = 0.0;
    if (tid == 0) ntot_s = 0.0;
    double gcur = 0.0, scur = 0.0, gnxt = 0.0, snxt = 0.0, ncur = 0.0, nnxt = 0.0;
    auto fetch = [&](int64_t sg, double (&v)[kPoolPer], double& gr, double& sh, double& n) {
        const double* G = gram + sg * q2;
#pragma unroll
        for (int k = 0; k < kPoolPer; ++k) v[k] = G[ro[k] * p2 + co[k]];
        n = G[0];
        if (tid < p2) {
            gr = G[tid];
            sh = shift[sg * p2 + tid];
        }
    };
    if (s0 < s1) fetch(s0, cur, gcur, scur, ncur);
    __syncthreads();
    for (int64_t sg = s0; sg < s1; ++sg) {
        if (sg + 1 < s1) fetch(sg + 1, nxt, gnxt, snxt, nnxt);
        const double nb = ncur;
        if (nb > 0) {                                  // uniform
            if (tid < p2 && tid > 0) {
                g0[tid] = gcur;
                dl[tid] = (scur + gcur / nb) - mu[tid];
            }
            if (tid == 0) {
                const double na = ntot_s;
                fac_s = na * nb / (na + nb);
                ntot_s = na + nb;
            }
            __syncthreads();
            const double fac = fac_s, ntot = ntot_s;   // (tid 0 rewrites them next segment)
#pragma unroll
            for (int k = 0; k < kPoolPer; ++k) {
                const int r = ro[k], c = co[k];
                const double cb = cur[k] - g0[r] * g0[c] / nb;             // segment centered
                acc[k] = acc[k] + cb + dl[r] * dl[c] * fac;
            }
            __syncthreads();
            if (tid < p2 && tid > 0) mu[tid] = mu[tid] + dl[tid] * (nb / ntot);
        }
#pragma unroll
        for (int k = 0; k < kPoolPer; ++k) cur[k] = nxt[k];
        gcur = gnxt;
        scur = snxt;
        ncur = nnxt;
    }
    __syncthreads();                                   // the last mu update
    double* og = out_gram + (int64_t)blockIdx.x * q2;
#pragma unroll
    for (int k = 0; k < kPoolPer; ++k)
        if (ebase + tid + k * kThreads < nel) {
            og[ro[k] * p2 + co[k]] = acc[k];
            og[co[k] * p2 + ro[k]] = acc[k];
        }
    if (blockIdx.y == 0) {                             // row / column 0: n, zeros; the means
        const double ntot = ntot_s;
        for (int c = tid; c < p2; c += kThreads) {
            og[c] = c == 0 ? ntot : 0.0;
            if (c > 0) og[c * p2] = 0.0;
        }
        if (tid < p2) out_shift[(int64_t)blockIdx.x * p2 + tid] = (tid == 0) ? 0.0 : mu[tid];
    }
}

// workgroups per date block that split the lower triangle of a (p2 x p2) Gram
static unsigned pool_split(int p2) {
    const int nel = (p2 - 1) * p2 / 2;
    return (unsigned)((nel + kPoolPer * kThreads - 1) / (kPoolPer * kThreads));
}

// ---- predictions: pred[t][a] = beta0 + sum_j beta_j x_j (grid rows with a set mask bit) ------
// HBM-bound: 8 B per regressor per test cell.  The column offsets are staged once per workgroup
// in LDS and each lane issues kPredBatch independent plane loads before folding them into the
// sum in order (s = s + b_j x_j, j ascending: the same operations as a plain loop), so a wave keeps
// a batch of loads in flight instead of one dependent load per regressor.
constexpr int kPredBatch = 16;
__global__ __launch_bounds__(256) void predict_kernel(const double* base, int64_t col_stride,
                                                      int64_t lda, int64_t t0, int64_t nt,
                                                      const int32_t* cols, int p,
                                                      const double* beta, int64_t beta_stride,
                                                      const uint64_t* bits, int ycheck,
                                                      double* pred) {
    __shared__ int64_t coff[kMaxF];
    for (int j = threadIdx.x; j < p; j += 256) coff[j] = (int64_t)cols[j] * col_stride;
    __syncthreads();
    const int64_t a = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    const int64_t t = t0 + (int64_t)blockIdx.y * 4 + (threadIdx.x >> 6);
    if (t >= t0 + nt) return;
    const double* b = beta + (t - t0) * beta_stride;
    const double* cell = base + t * lda + a;
    u64 w = bits[(t >> 6) * lda + a];
    double v = __builtin_nan("");
    bool use = (w >> (t & 63)) & 1ull;
    if (use && ycheck >= 0) use = __builtin_isfinite(cell[(int64_t)ycheck * col_stride]);
    if (use) {
        double s = b[0];
        int j = 0;
        for (; j + kPredBatch <= p; j += kPredBatch) {
            double x[kPredBatch];
#pragma unroll
            for (int k = 0; k < kPredBatch; ++k) x[k] = cell[coff[j + k]];
#pragma unroll
            for (int k = 0; k < kPredBatch; ++k) s = s + b[1 + j + k] * x[k];
        }
        for (; j < p; ++j) s = s + b[1 + j] * cell[coff[j]];
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
    AFM_TAIL_PRIO_SET();
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

#ifdef AFM_FP_PROFILE
extern "C" int afm_debug_gram_cycles(long long* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(afm::g_gram_cycles), sizeof(long long) * n) ==
                   hipSuccess ? 0 : -1;
}
#endif

template <int NT>
static hipError_t launch_gram_nt(int mode, dim3 grid, hipStream_t st, const GramArgs& g) {
    const dim3 blk(512);
    switch (mode) {
        case 0: hipLaunchKernelGGL((gram_kernel<NT, 0>), grid, blk, 0, st, g); break;
        case 1: hipLaunchKernelGGL((gram_kernel<NT, 1>), grid, blk, 0, st, g); break;
        default: hipLaunchKernelGGL((gram_kernel<NT, 2>), grid, blk, 0, st, g); break;
    }
    return hipGetLastError();
}

static hipError_t launch_gram(int nt, int mode, dim3 grid, hipStream_t st, const GramArgs& g) {
    switch (nt) {
        case 1: return launch_gram_nt<1>(mode, grid, st, g);
        case 2: return launch_gram_nt<2>(mode, grid, st, g);
        case 3: return launch_gram_nt<3>(mode, grid, st, g);
        case 4: return launch_gram_nt<4>(mode, grid, st, g);
        case 5: return launch_gram_nt<5>(mode, grid, st, g);
        case 6: return launch_gram_nt<6>(mode, grid, st, g);
        default: return launch_gram_nt<7>(mode, grid, st, g);
    }
}

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
    const int nt = (p + 15) / 16;
    // option gram_checked: the checked staging only (A/B tests)
    const bool checked = ctx->gram_checked != 0;
    for (const int mode : {checked ? 0 : 1, checked ? -1 : 2}) {
        if (mode < 0) break;
        AFM_HIP(launch_gram(nt, mode, dim3((unsigned)nseg), ctx->stream, g));
    }
    return AFM_OK;
}

extern "C" int afm_ols_solve_f64(afm_ctx* ctx, const double* gram, const double* shift, int p,
                                 int64_t nseg, double tol, double* beta, double* nobs,
                                 int32_t* rank) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(p >= 1 && p <= kMaxP, "need 1 <= p <= 110");
    AFM_CHECK_ARG(gram && shift && beta && nobs && rank, "null buffer");
    if (nseg <= 0) return AFM_OK;
    SolveArgs s{gram, shift, p, tol, nullptr, p, beta, nobs, rank};
    const size_t lds = sizeof(double) * (size_t)(p + 1) * (p + 2) / 2;     // packed triangle
    AFM_HIP(afm_lds_opt_in(ctx, (const void*)ols_solve_kernel, (int)lds));
    hipLaunchKernelGGL(ols_solve_kernel, dim3((unsigned)nseg), dim3(kThreads), lds, ctx->stream,
                       s);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

// The pooling tree: level 0 merges 16 consecutive segments (dates), level 1 four level-0
// results (64-date blocks), every later level 8 results, until one is left.  Each level is one
// pool_kernel launch whose chains are at most 16 merges long (the former two-pass tree ran 64 +
// 63 sequential merges).  The tree is a fixed function of the segment list, so any split of the
// dates into 64-aligned ranges (multi-GPU) reproduces it: a rank pools its own dates through
// levels 0-1 and the gathered 64-date blocks go through levels 2+ (afm_pool_tree_f64).
static int64_t pool_level_per(int level) { return level == 0 ? 16 : level == 1 ? 4 : 8; }

static int pool_tree(afm_ctx* ctx, const double* gram, const double* shift, int p, int64_t nseg,
                     int level0, double* out_gram, double* out_shift) {
    const int p2 = p + 2;
    const unsigned ny = pool_split(p2);
    // (a level over one segment is an exact identity merge: from n = 0 the Chan factor is 0)
    auto blocks = [](int64_t n, int64_t per) -> int64_t {
        return n <= per ? 1 : (n + per - 1) / per;
    };
    const int64_t nb0 = blocks(nseg, pool_level_per(level0));
    double* work = nullptr;
    if (nb0 > 1) {
        hipError_t e;
        work = (double*)afm_ctx_scratch(ctx, AFM_SCRATCH_POOL,
                                        sizeof(double) * 2 * nb0 * (p2 * p2 + p2), &e);
        AFM_HIP(e);
    }
    const double* ig = gram;
    const double* is = shift;
    int64_t n = nseg;
    for (int level = level0, pp = 0;; ++level, pp ^= 1) {
        const int64_t per = pool_level_per(level);
        const int64_t nb = blocks(n, per);
        double* og = nb == 1 ? out_gram : work + pp * nb0 * (p2 * p2 + p2);
        double* os = nb == 1 ? out_shift : og + nb0 * p2 * p2;
        hipLaunchKernelGGL(pool_kernel, dim3((unsigned)nb, ny), dim3(kThreads), 0, ctx->stream, ig,
                           is, p2, n, per, og, os);
        AFM_HIP(hipGetLastError());
        if (nb == 1) break;
        ig = og;
        is = os;
        n = nb;
    }
    return AFM_OK;
}

extern "C" int afm_pool_moments_f64(afm_ctx* ctx, const double* gram, const double* shift, int p,
                                    int64_t nseg, double* out_gram, double* out_shift) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(p >= 1 && p + 2 <= kMaxF, "need 1 <= p <= 110");
    AFM_CHECK_ARG(gram && shift && out_gram && out_shift && nseg >= 0, "bad arguments");
    return pool_tree(ctx, gram, shift, p, nseg, 0, out_gram, out_shift);
}

extern "C" int afm_pool_tree_f64(afm_ctx* ctx, const double* gram, const double* shift, int p,
                                 int64_t nseg, int level0, double* out_gram, double* out_shift) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(p >= 1 && p + 2 <= kMaxF, "need 1 <= p <= 110");
    AFM_CHECK_ARG(gram && shift && out_gram && out_shift && nseg >= 0 && level0 >= 0,
                  "bad arguments");
    return pool_tree(ctx, gram, shift, p, nseg, level0, out_gram, out_shift);
}

extern "C" int afm_pool_segments_f64(afm_ctx* ctx, const double* gram, const double* shift,
                                     int p, int64_t nseg, int64_t per, double* out_gram,
                                     double* out_shift) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(p >= 1 && p + 2 <= kMaxF, "need 1 <= p <= 110");
    AFM_CHECK_ARG(gram && shift && out_gram && out_shift && nseg >= 0 && per >= 1, "bad arguments");
    if (nseg == 0) return AFM_OK;
    const int p2 = p + 2;
    const int64_t nb = (nseg + per - 1) / per;
    hipLaunchKernelGGL(pool_kernel, dim3((unsigned)nb, pool_split(p2)), dim3(kThreads), 0,
                       ctx->stream, gram, shift, p2, nseg, per, out_gram, out_shift);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_predict_f64(afm_ctx* ctx, const double* base, int64_t col_stride, int64_t lda,
                               int64_t t0, int64_t nt, const int32_t* cols, int p,
                               const double* beta, int64_t beta_stride, const uint64_t* bits,
                               int ycheck, double* pred) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(base && cols && beta && bits && pred, "null buffer");
    AFM_CHECK_ARG(lda % 64 == 0 && nt >= 0 && t0 >= 0, "bad shape");
    AFM_CHECK_ARG(p >= 0 && p <= kMaxF, "need 0 <= p <= 112");
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

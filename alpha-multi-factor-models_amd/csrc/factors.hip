// Factor panel: the 98 output columns of No-talib.py:1-93 for a
// calendar-grid panel, bit-exact with pandas 2.3.3.
//
// Layout (include/afm.h): inputs [T][lda] fp64 date-major/asset-minor, presence bits
// [ceil(T/64)][lda] uint64, output planes [98][T][lda].
//
// Kernel design (MI355X):
//  * pandas' rolling/ewm kernels are sequential recurrences whose rounding depends on the full
//    history (Kahan compensations are never reset), so bit-exactness requires a sequential scan
//    per asset.  Parallelism = assets (one per lane) x indicator jobs (one job set per wave).
//  * One 64-asset block = 15 job waves (balanced by the VALU count of each job's compiled step,
//    and so that the four SIMDs carry equal totals) + a loader wave per item.  At config C the
//    kernel is bound by its output stream in this pattern (~4.7 TB/s; without the stores it runs
//    in ~2/3 of the time) beside the f64 VALU work; at small shards by the longest job set's
//    dependency chain.  An LDS ring holds the last kRing present observations of
//    close and volume per lane.  A shard with few blocks (multi-GPU)
//    splits each block's 15 job waves over 3, 5 or 15 workgroups instead, so that ~all CUs work
//    (each split needs its own ring; measured on MI355X, workgroups of 78 KB LDS do not
//    co-reside -- the two-per-CU limit was between 52 and 56 KB -- hence one per CU).
//  * The loader wave is the only one that reads global memory: it fills the ring one chunk
//    ahead of the scan and publishes each chunk's presence bits.  The job waves only store, so
//    they never wait on vmcnt (loads and stores share the counter on gfx950: a wave that both
//    prefetches and streams stores must drain its stores before it can use a prefetched value).
//  * Windows are positional over each asset's PRESENT days (holes and listing gaps do not count,
//    No-talib.py:5-6); the ring is indexed by the lane's observation count (mod kRing).
//  * Time advances in chunks of kChunk = 8 calendar days, one barrier per chunk: the job waves
//    step their jobs over chunk c's present days and stream their output columns (16-B stores of
//    two columns, see lane_asset) while the loader writes chunk c+1 into the ring and issues the
//    loads of chunk c+2.  Cells of absent asset-days in a date row the wave writes hold NaN.
//    (Round 4 measured a barrier-free hand-off -- LDS counters, 4- or 8-day chunks, up to 3
//    chunks of skew between job waves: 11.6-11.9 vs 10.6-10.8 ms at config C)
//  * Divisions by an observation count (window means, Welford updates, variances, PSY) use a
//    correctly rounded reciprocal table and one Markstein correction -- the exactly rounded
//    quotient for every integer divisor <= 64 (FMA; no contraction elsewhere); ewm skips its
//    division by (old + alpha) == 1.0 exactly.  Other divisions are IEEE.
//  * dropna bookkeeping: each job wave keeps its per-lane "some output NaN / non-finite at day s"
//    bits and stores them at each 64-day word; masks_kernel ORs the partials into
//    nanfree / finite.
//
// Algorithmic traffic per present asset-day: 32 B of inputs read + 98 x 8 B written = 816 B.
#include "afm_internal.h"

#include <type_traits>

#include <cstdlib>

#pragma clang fp contract(off)

namespace afm {
namespace {

constexpr int kLanes = 64;
constexpr int kChunk = 8;
// the loader fills chunk c+1 while the job waves scan chunk c: the ring must hold the scan's
// lookback (57) plus two chunks
constexpr int kRing = 57 + 2 * kChunk + 1;

typedef unsigned long long u64;
#ifdef AFM_FP_PROFILE
// profiling build only: per-(workgroup, wave) cycles spent in the chunk loop
__device__ long long g_wave_cycles[1 << 16];
#endif
// explicit address spaces: the per-wave functions are not inlined, and generic (flat) pointers
// would turn every ring read into a flat_load that waits on all outstanding global stores
#define LDS __attribute__((address_space(3)))
#define GLB __attribute__((address_space(1)))

__device__ __forceinline__ double qnan() { return __builtin_nan(""); }
// Workgroup barrier ordering LDS only: the ring and the NaN masks live in LDS; the output stores
// need no ordering, so the barrier must not wait for them (__syncthreads() waits vmcnt(0)).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ double pinf(double x) { return __builtin_isinf(x) ? qnan() : x; }
// pandas zsqrt: negative -> 0, NaN stays NaN
__device__ __forceinline__ double zsqrt(double x) { return x < 0 ? 0.0 : __builtin_sqrt(x); }

struct Smem {
    double c[kRing][kLanes];   // close ring (by observation index mod kRing)
    double v[kRing][kLanes];   // volume ring
    double rtab[128];          // rtab[n] = 1.0 / n (IEEE), rtab[0] = +inf; indexed n & 127
    int cbyte[2][kLanes];      // presence bits of chunk c (parity c & 1), written by the loader
    int okbyte[2][kLanes];     // chunk c: 2 every present day clean (kClean), 1 warm, 0 general
};
// The small-grid partition (PartS below) adds, per workgroup:
//  * rings of close.pct_change() and volume.pct_change() per observation (by observation index
//    mod kRingR), computed ONCE by the loader -- the job waves read the returns / volume changes
//    at any lookback instead of dividing (every return-based job: sd_*, corr_*, PVT);
//  * the exchange of the split rolling correlations: for chunk c (parity c & 1) the numerator
//    wave writes num, the denominator wave den, per present day; a combining wave forms
//    num / den for chunk c during chunk c + 1 (after the barrier between them).
// 140 KB: one workgroup per CU (the launch sizes its grid to <= the CU count).
constexpr int kRingR = 32;           // lookbacks 0..15 + two chunks of look-ahead
constexpr int kXSlots = 2;           // exchange slots of one workgroup
// Combiner kinds (Comb<K>): the column num / den of the previous chunk -- 0: corr_5, 1: corr_15
// (PartS, PartT), 2: sd5_15, 3: volsd5_15 (PartT); kind k uses exchange slot k & 1, so a workgroup
// may hold kinds 0 and 1, or 2 and 3 (the partitions place them so)
constexpr int kCombs = 4;
constexpr int comb_col(int k) { return k == 0 ? 94 : k == 1 ? 95 : k == 2 ? 88 : 92; }
constexpr int comb_slot(int k) { return k & 1; }
struct SmemRG : Smem {
    double r[kRingR][kLanes];
    double g[kRingR][kLanes];
    double xnum[kXSlots][2][kChunk][kLanes];
    double xden[kXSlots][2][kChunk][kLanes];
};

// ---- clean windows ----------------------------------------------------------------------------
// A present day is CLEAN when it and the kClean - 1 observations before it all have close and
// volume in (kLo, kHi).  Over a clean day every job's inputs are finite and non-NaN (no NaN skip
// fires, every window holds exactly W observations, close / volume / volume*close windows hold no
// negative value, no sum or product overflows), so the pandas recurrences reduce to their
// branch-free cores with compile-time counts.  A chunk whose present days are clean for all 64
// lanes of the wave runs the fast step (fstep); any other chunk runs the general step.  Both
// perform the same IEEE operations on the same states, so the results are bit-identical.
constexpr int kClean = 58;           // ACCEL_56 reads close 57 observations back
constexpr double kLo = 1e-50, kHi = 1e50;

// x / n exactly rounded for integer 0 <= n <= 64 (Markstein: r = RN(1/n), q0 = RN(x r),
// q = RN(q0 + (x - q0 n) r)); zero and non-finite quotients pass through (keeps -0, inf, NaN).
// Out-of-range n (only in discarded lanes of the branch-free updates) reads a defined entry.
__device__ __forceinline__ double div_n(const LDS Smem* sm, double x, int n) {
    const double d = (double)n;
    const double r = sm->rtab[n & 127];
    const double q0 = x * r;
    const double e = __builtin_fma(-q0, d, x);
    const double q1 = __builtin_fma(e, r, q0);
    return (q0 == 0.0 || !__builtin_isfinite(q0)) ? q0 : q1;
}
// The same quotient for a compile-time divisor and an x that is finite and not -0 (every clean
// window sum, Welford increment and sum of squares: they start at +0 and RN addition never
// yields -0 from operands that are not both -0).  For x = +0 the Markstein steps return +0.
template <int N>
__device__ __forceinline__ double divc(double x) {
    constexpr double r = 1.0 / (double)N;
    const double q0 = x * r;
    const double e = __builtin_fma(-q0, (double)N, x);
    return __builtin_fma(e, r, q0);
}

struct Args {
    int64_t T, lda, plane;     // plane = T * lda
    const GLB double* close;
    const GLB double* volume;
    const GLB uint64_t* vbits;
    GLB double* out;
    GLB uint64_t* nanpart;     // [nparts][words][lda] per-job-wave "some output NaN" bits
    GLB uint64_t* badpart;     // [nparts][words][lda] per-job-wave "some output non-finite" bits
    GLB uint64_t* cnanpart;    // (kernel-set) the split correlations' combiner partials
    GLB uint64_t* cbadpart;
    int64_t pstride;           // (kernel-set) words * lda: one partial's plane
    int jw;                    // profiling build: job waves per item
    int types;                 // workgroups per 64-asset block (1, 3, 5 or 15)
    int fast;                  // 0: general step only (A/B tests)
    int nblk;                  // 64-asset blocks (paired launch: items = nblk * types)
    int pslot;                 // profiling build: block * types + type of the running item
    // time slab [c0 * kChunk, t1) (c0 * kChunk a multiple of 64): out and the mask partials hold
    // only the slab's dates (out is offset by the host so that date t's row is out + t * lda);
    // state (or null) carries every wave's recurrence state and the loaders' rings across slabs
    int c0, c1;                // chunk range of the slab
    int64_t t1;                // slab end (exclusive)
    GLB double* state;         // [nblk][types][jobs + 1][kStateWords][64]
    int load_state;            // the slab continues a series: restore the state first
};

// Ring cell of lookback L (observation p - L) as a byte offset from row 0, given pmoff = the
// byte offset of (row pm = p mod kRing, this lane): the unsigned min of (pm - L) and
// (pm - L + kRing) rows -- the first wraps to a huge value exactly when pm < L.
__device__ __forceinline__ uint32_t ring_off(uint32_t pmoff, int L) {
    const uint32_t a = pmoff - (uint32_t)(L * kLanes * 8);
    const uint32_t b = pmoff + (uint32_t)((kRing - L) * kLanes * 8);
    return a < b ? a : b;
}

// Per-series run of equal consecutive values (pandas roll_mean / roll_var "same value" rule):
// identical for every window over the same series, so it is kept once per series and wave.
struct Run {
    double prev;
    int same;
    __device__ __forceinline__ void init() { prev = qnan(); same = 0; }
    __device__ __forceinline__ void upd(double x) {          // NaN values are skipped
        if (x == x) {
            same = (x == prev) ? same + 1 : 1;
            prev = x;
        }
    }
    __device__ __forceinline__ void fupd(double x) {         // x known non-NaN
        same = (x == prev) ? same + 1 : 1;
        prev = x;
    }
};
// C close, V volume, VP pinf(volume), VC pinf(volume * close), R pinf(ret), X / Y / XY the
// rolling-corr pair (pinf(ret + 0 vol_change), pinf(vol_change + 0 ret), X * Y).
struct Runs {
    Run C, V, VP, VC, R, X, Y, XY;
};

// ---- output stores --------------------------------------------------------------------------
// Lanes and assets (round 4): lane i < 32 holds asset 2i of its 64-asset block, lane i + 32 asset
// 2i + 1 (lane_asset).  A step's output values are stored two columns at a time: after
// v_permlane32_swap of the two values, lane i holds BOTH assets of the first column and lane
// i + 32 both assets of the second, so one 16-B store per lane writes 512 contiguous bytes of
// each column's row -- half the store instructions of one 8-B store per column (at config C the
// kernel is bound by its write stream meeting the recurrences).  The stores run
// with the whole wave active after the day's (divergent) step: a lane absent that day writes NaN
// into its cells.
__device__ __forceinline__ int lane_asset(int lane) { return 2 * (lane & 31) + (lane >> 5); }

// the columns a job writes, as a 96-bit mask (lo: columns 0-63, hi: 64-95)
struct Cols {
    u64 lo, hi;
};
constexpr Cols col1(int c) { return c < 64 ? Cols{1ull << c, 0} : Cols{0, 1ull << (c - 64)}; }
constexpr Cols operator|(Cols a, Cols b) { return Cols{a.lo | b.lo, a.hi | b.hi}; }
constexpr int ncols(Cols m) { return __builtin_popcountll(m.lo) + __builtin_popcountll(m.hi); }
struct ColList {
    int c[96];
};
constexpr ColList col_list(Cols m) {
    ColList l{};
    int n = 0;
    for (int c = 0; c < 96; ++c)
        if (c < 64 ? ((m.lo >> c) & 1ull) : ((m.hi >> (c - 64)) & 1ull)) l.c[n++] = c;
    return l;
}

// Per-lane view of one (asset, present day) step.  Lookback L reads observation p - L.
// RG: the workgroup has the loader's return / volume-change rings (SmemRG).
template <bool RG>
struct Step {
    static constexpr bool kRG = RG;
    const LDS Smem* sm;
    GLB double* out;           // output row of this day: a.out + t * lda (uniform)
    Runs* rn;
    int64_t plane;
    uint32_t voff, pmoff;      // asset * 8; (pm * kLanes + lane) * 8 (pm = p mod kRing)
    uint32_t p32off;           // RG: ((p mod kRingR) * kLanes + lane) * 8
    int sday, par;             // the day's index in its chunk; the chunk's parity
    uint32_t poff;             // (block * 64 + 2 * (lane & 31)) * 8: the lane's asset pair
    int64_t hmask;             // lane >= 32 ? -1 : 0
    int lane, p;
    bool anynan, anybad;
    double r0, g0;             // ret(p), vol_change(p), computed once per step when needed
    double ov[96];             // the step's output values by column (only the pack's are used)
    __device__ __forceinline__ double C(int L) const {
        return *(const LDS double*)((const LDS char*)&sm->c[0][0] + ring_off(pmoff, L));
    }
    __device__ __forceinline__ double V(int L) const {
        return *(const LDS double*)((const LDS char*)&sm->v[0][0] + ring_off(pmoff, L));
    }
    // RG: return / volume change of observation p - L (NaN for observation 0), L < 16
    __device__ __forceinline__ uint32_t rg_off(int L) const {
        return (p32off - (uint32_t)(L * kLanes * 8)) & (uint32_t)(kRingR * kLanes * 8 - 1);
    }
    __device__ __forceinline__ double Rr(int L) const {
        return *(const LDS double*)((const LDS char*)&((const LDS SmemRG*)sm)->r[0][0] + rg_off(L));
    }
    __device__ __forceinline__ double Gr(int L) const {
        return *(const LDS double*)((const LDS char*)&((const LDS SmemRG*)sm)->g[0][0] + rg_off(L));
    }
    __device__ __forceinline__ double div(double x, int n) const { return div_n(sm, x, n); }
    __device__ __forceinline__ void put(int col, double x) {
        ov[col] = x;
        anynan |= (x != x);
        anybad |= !__builtin_isfinite(x);
    }
    // fast step: columns that are finite on a clean day need no NaN / inf bookkeeping
    __device__ __forceinline__ void putf(int col, double x) { ov[col] = x; }
    // before the day's step: the pack's columns NaN (what an absent lane stores)
    template <u64 LO, u64 HI>
    __device__ __forceinline__ void reset() {
        constexpr Cols m{LO, HI};
        constexpr int n = ncols(m);
        constexpr ColList l = col_list(m);
#pragma unroll
        for (int k = 0; k < n; ++k) ov[l.c[k]] = qnan();
    }
    // one column, 8 B per lane: a buffer_store with an SGPR descriptor based at the column row and
    // the lane's 32-bit byte offset (the scheduler may place it anywhere after its value; raw
    // buffer, num_records bounds the offset; word 3 = 0x00020000, the CDNA raw-buffer format)
    __device__ __forceinline__ void store1(int col, double x) {
        typedef unsigned v2u __attribute__((ext_vector_type(2)));
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(out + col * plane), 0, 0x7fffffff, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, x), r, (int)voff, 0, 0);
    }
    // two columns, 16 B per lane (see lane_asset)
    __device__ __forceinline__ void store2(int c1, double x1, int c2, double x2) {
        typedef unsigned v2u __attribute__((ext_vector_type(2)));
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        const v2u a = __builtin_bit_cast(v2u, x1), b = __builtin_bit_cast(v2u, x2);
        const auto l = __builtin_amdgcn_permlane32_swap(a.x, b.x, false, false);
        const auto h = __builtin_amdgcn_permlane32_swap(a.y, b.y, false, false);
        const v4u w = {l[0], h[0], l[1], h[1]};
        // the upper half-wave's row: the first column's row + (c2 - c1) planes (uniform), masked
        const int64_t d = (int64_t)(c2 - c1) * plane * 8;
        GLB char* row = (GLB char*)(out + c1 * plane) + (d & hmask);
        *(GLB v4u*)(row + poff) = w;
    }
    // after the day's step, the whole wave active: the pack's columns in pairs
    template <u64 LO, u64 HI>
    __device__ __forceinline__ void flush() {
        constexpr Cols m{LO, HI};
        constexpr int n = ncols(m);
        constexpr ColList l = col_list(m);
#pragma unroll
        for (int k = 0; k + 1 < n; k += 2) store2(l.c[k], ov[l.c[k]], l.c[k + 1], ov[l.c[k + 1]]);
        if constexpr ((n & 1) != 0) store1(l.c[n - 1], ov[l.c[n - 1]]);
    }
    // close.pct_change() at lookback L (p - L >= 0), NaN for observation 0
    __device__ __forceinline__ double ret(int L) const {
        if (L == 0) return r0;
        if constexpr (RG) return Rr(L);
        const double r = C(L) / C(L + 1) - 1;
        return p - L >= 1 ? r : qnan();
    }
    __device__ __forceinline__ double volchg(int L) const {
        if (L == 0) return g0;
        if constexpr (RG) return Gr(L);
        const double g = V(L) / V(L + 1) - 1;
        return p - L >= 1 ? g : qnan();
    }
};

// A clean or warm step's view (see kClean): every ring value the wave's jobs read, gathered at the
// top of the step in one batch of LDS reads (CM / VM: bit L = lookback L of close / volume), so
// the step waits for LDS once instead of once per job.  A job reads a lookback its pack did not
// gather only by a compile error.
constexpr int kLook = 58;            // lookbacks 0 .. 57 (ACCEL_56 reads close 57 back)
// s_waitcnt vmcnt(0) with expcnt / lgkmcnt left at their maxima (gfx9 encoding)
constexpr int kWaitVm0 = 0x0f70;
template <bool RG, u64 CM, u64 VM, u64 RM, u64 GM>
struct FastStep : Step<RG> {
    // RM / GM: the return / volume-change lookbacks the pack reads (RG: from the rings; else
    // divided from the close / volume lookbacks L, L + 1, which CM / VM then include)
    double cc[kLook], vc[kLook], rr[16], gg[16];
    __device__ __forceinline__ void gather() {
#pragma unroll
        for (int L = 0; L < kLook; ++L) {
            if ((CM >> L) & 1ull) cc[L] = this->C(L);
            if ((VM >> L) & 1ull) vc[L] = this->V(L);
        }
        if constexpr (RG) {
#pragma unroll
            for (int L = 0; L < 16; ++L) {
                if ((RM >> L) & 1ull) rr[L] = this->Rr(L);
                if ((GM >> L) & 1ull) gg[L] = this->Gr(L);
            }
        }
    }
    template <int L>
    __device__ __forceinline__ double c() const {
        static_assert(L < kLook && ((CM >> L) & 1ull), "close lookback not gathered");
        return cc[L];
    }
    template <int L>
    __device__ __forceinline__ double v() const {
        static_assert(L < kLook && ((VM >> L) & 1ull), "volume lookback not gathered");
        return vc[L];
    }
    // return / volume change at lookback L on a clean day (every observation finite)
    template <int L>
    __device__ __forceinline__ double fret() const {
        static_assert(L < 16 && ((RM >> L) & 1ull), "return lookback not declared");
        if constexpr (L == 0) return this->r0;        // computed once per step (run_wave)
        else if constexpr (RG) return rr[L];
        else return c<L>() / c<L + 1>() - 1;
    }
    template <int L>
    __device__ __forceinline__ double fvolchg() const {
        static_assert(L < 16 && ((GM >> L) & 1ull), "volume-change lookback not declared");
        if constexpr (L == 0) return this->g0;
        else if constexpr (RG) return gg[L];
        else return v<L>() / v<L + 1>() - 1;
    }
};
constexpr u64 lb(int L) { return 1ull << L; }
#define FC(L) s.template c<(L)>()
#define FV(L) s.template v<(L)>()

// ---- pandas window kernels as register-resident recurrences -------------------------------
// roll_mean (pandas/_libs/window/aggregations.pyx): Kahan add/remove with separate
// compensations, same-value run rule (Run), sign rules.
struct RollMean {
    double sum, cadd, crem;
    int nobs, neg;
    __device__ __forceinline__ void init() {
        sum = cadd = crem = 0.0;
        nobs = neg = 0;
    }
    __device__ __forceinline__ void add(double x) {
        if (x == x) {
            nobs++;
            double y = x - cadd, t = sum + y;
            cadd = t - sum - y;
            sum = t;
            neg += __builtin_signbit(x) ? 1 : 0;
        }
    }
    __device__ __forceinline__ void remove(double x) {
        if (x == x) {
            nobs--;
            double y = -x - crem, t = sum + y;
            crem = t - sum - y;
            sum = t;
            neg -= __builtin_signbit(x) ? 1 : 0;
        }
    }
    template <class S>
    __device__ __forceinline__ double result(const S& s, int minp, const Run& rn) const {
        if (nobs >= minp && nobs > 0) {
            double r = s.div(sum, nobs);
            if (rn.same >= nobs) r = rn.prev;
            else if (neg == 0 && r < 0) r = 0.0;
            else if (neg == nobs && r > 0) r = 0.0;
            return r;
        }
        return qnan();
    }
    // clean window: the Kahan cores only (nobs stays W)
    __device__ __forceinline__ void fremove(double x) {
        double y = -x - crem, t = sum + y;
        crem = t - sum - y;
        sum = t;
    }
    __device__ __forceinline__ void fadd(double x) {
        double y = x - cadd, t = sum + y;
        cadd = t - sum - y;
        sum = t;
    }
    // a window of positive values: neg = 0 < W, so only the "negative mean -> 0" rule can fire;
    // the mean is never NaN or -0 here, so it is a max with +0
    template <int W>
    __device__ __forceinline__ double fresult_pos(const Run& rn) const {
        const double r = __builtin_fmax(divc<W>(sum), 0.0);
        return rn.same >= W ? rn.prev : r;
    }
    // a signed series: the sign counts are kept
    __device__ __forceinline__ void fsigns(double xadd, double xrem) {
        neg += (__builtin_signbit(xadd) ? 1 : 0) - (__builtin_signbit(xrem) ? 1 : 0);
    }
    // warm window (see "warm-up windows" below): the Kahan cores, remove value 0 before the window
    // is full (exactly a no-op while crem is still +0), the count kept for the general step
    __device__ __forceinline__ void wstep(double xrem, double xadd, int n) {
        fremove(xrem);
        fadd(xadd);
        nobs = n;
    }
    template <int W>
    __device__ __forceinline__ double fresult(const Run& rn) const {
        double r = divc<W>(sum);
        if (rn.same >= W) r = rn.prev;
        else if (neg == 0 && r < 0) r = 0.0;
        else if (neg == W && r > 0) r = 0.0;
        return r;
    }
};

// roll_var, ddof = 1: Welford with Kahan-compensated mean; the remove runs before the add.
struct RollVar {
    double mean, ssq, cadd, crem;
    int nobs;
    __device__ __forceinline__ void init() {
        mean = ssq = cadd = crem = 0.0;
        nobs = 0;
    }
    template <class S>
    __device__ __forceinline__ void add(const S& s, double x) {
        if (!__builtin_isnan(x)) {
            nobs = nobs + 1;
            double pm = mean - cadd, y = x - cadd, t = y - mean;
            cadd = t + mean - y;
            mean = mean + s.div(t, nobs);
            ssq = ssq + (x - pm) * (x - mean);
        }
    }
    template <class S>
    __device__ __forceinline__ void remove(const S& s, double x) {
        if (!__builtin_isnan(x)) {
            nobs = nobs - 1;
            if (nobs != 0) {
                double pm = mean - crem, y = x - crem, t = y - mean;
                crem = t + mean - y;
                mean = mean - s.div(t, nobs);
                ssq = ssq - (x - pm) * (x - mean);
            } else {
                mean = 0.0;
                ssq = 0.0;
            }
        }
    }
    template <class S>
    __device__ __forceinline__ double result(const S& s, int minp, const Run& rn) const {
        if (nobs >= minp && nobs > 1)
            return (rn.same >= nobs) ? 0.0 : s.div(ssq, nobs - 1);
        return qnan();
    }
    // clean window of W: nobs W -> W - 1 -> W
    template <int W>
    __device__ __forceinline__ void fremove(double x) {
        double pm = mean - crem, y = x - crem, t = y - mean;
        crem = t + mean - y;
        mean = mean - divc<W - 1>(t);
        ssq = ssq - (x - pm) * (x - mean);
    }
    template <int W>
    __device__ __forceinline__ void fadd(double x) {
        double pm = mean - cadd, y = x - cadd, t = y - mean;
        cadd = t + mean - y;
        mean = mean + divc<W>(t);
        ssq = ssq + (x - pm) * (x - mean);
    }
    template <int W>
    __device__ __forceinline__ double fresult(const Run& rn) const {
        return (rn.same >= W) ? 0.0 : divc<W - 1>(ssq);
    }
    // warm add: the count n = nobs after the add (1 .. W) varies per lane while the window fills
    template <class S>
    __device__ __forceinline__ void wadd(const S& s, double x, int n) {
        double pm = mean - cadd, y = x - cadd, t = y - mean;
        cadd = t + mean - y;
        mean = mean + s.div(t, n);
        ssq = ssq + (x - pm) * (x - mean);
        nobs = n;
    }
};

// ewm(adjust=False, ignore_na=False).mean(), minp = 1.  wtd starts NaN / old = 1, which
// reproduces pandas' special first element exactly.  pandas emits wtd once nobs >= 1; wtd is
// NaN exactly until the first observation, so the emitted value is wtd itself.
// (old + alpha) is 1.0 exactly after every observed step for the spans/coms used here; the
// division by it is then the identity and is skipped (bit-identical).
struct Ewm {
    double wtd, old;
    __device__ __forceinline__ void init() {
        wtd = qnan();
        old = 1.0;
    }
    __device__ __forceinline__ double step(double cur, double owf, double nw) {
        bool obs = (cur == cur);
        if (wtd == wtd) {
            old *= owf;
            if (obs) {
                if (wtd != cur) {
                    const double num = old * wtd + nw * cur;
                    const double den = old + nw;
                    wtd = num;
                    if (den != 1.0) wtd = num / den;
                }
                old = 1.0;
            }
        } else if (obs) {
            wtd = cur;
        }
        return wtd;
    }
    // clean step: the previous day was observed, so old = 1 on entry (and again on exit), wtd is
    // not NaN (an observed day after a NaN weight resets it) and old * owf = owf; owf + nw == 1
    __device__ __forceinline__ double fstep(double cur, double owf, double nw) {
        const double num = owf * wtd + nw * cur;
        wtd = (wtd != cur) ? num : wtd;
        return wtd;
    }
    // warm step of a series observed on every present day from `first` on (cur finite there):
    // before it wtd stays NaN, at it wtd = cur (pandas' first element), then the clean step
    __device__ __forceinline__ double wstep(double cur, double owf, double nw, int p, int first) {
        const double num = owf * wtd + nw * cur;
        const double f = (wtd != cur) ? num : wtd;
        wtd = p > first ? f : (p == first ? cur : wtd);
        return wtd;
    }
};

// alpha = 1 / (1 + com) exactly as pandas computes it (constant-folded in IEEE double)
template <int SPAN>
struct SpanC {
    static constexpr double com = (SPAN - 1) / 2.0;
    static constexpr double alpha = 1.0 / (1.0 + com);
    static constexpr double owf = 1.0 - alpha;
    static_assert(owf + alpha == 1.0, "ewm fast step needs (1 - alpha) + alpha == 1");
};
template <int COM>
struct ComC {
    static constexpr double alpha = 1.0 / (1.0 + (double)COM);
    static constexpr double owf = 1.0 - alpha;
    static_assert(owf + alpha == 1.0, "ewm fast step needs (1 - alpha) + alpha == 1");
};

// ---- jobs (one output group each; columns in No-talib.py order, see abi.cpp) --------------
// step(): any day (pandas semantics in full); fstep(): a clean day (see kClean).
template <int W>
struct Sma {  // No-talib.py:9-10
    static constexpr u64 kC = lb(0) | lb(W), kV = 0;
    static constexpr u64 kRt = 0, kGc = 0;
    static constexpr Cols kOut = col1((W - 6) / 4);
    RollMean m;
    __device__ void init() { m.init(); }
    template <class S> __device__ void step(S& s) {
        if (s.p >= W) m.remove(s.C(W));
        m.add(s.C(0));
        s.put((W - 6) / 4, m.result(s, W, s.rn->C));
    }
    template <class S> __device__ void fstep(S& s) {
        m.fremove(FC(W));
        m.fadd(FC(0));
        s.putf((W - 6) / 4, m.fresult_pos<W>(s.rn->C));
    }
    template <class S> __device__ void wstep(S& s) {
        m.wstep(s.p >= W ? FC(W) : 0.0, FC(0), s.p >= W ? W : s.p + 1);
        const double r = m.fresult_pos<W>(s.rn->C);
        s.putf((W - 6) / 4, s.p >= W - 1 ? r : qnan());
    }
};

template <int W>
struct Ema {  // No-talib.py:13-14
    static constexpr u64 kC = lb(0), kV = 0;
    static constexpr u64 kRt = 0, kGc = 0;
    static constexpr Cols kOut = col1(12 + (W - 6) / 4);
    Ewm e;
    __device__ void init() { e.init(); }
    template <class S> __device__ void step(S& s) {
        s.put(12 + (W - 6) / 4, e.step(s.C(0), SpanC<W>::owf, SpanC<W>::alpha));
    }
    template <class S> __device__ void fstep(S& s) {
        s.putf(12 + (W - 6) / 4, e.fstep(FC(0), SpanC<W>::owf, SpanC<W>::alpha));
    }
    template <class S> __device__ void wstep(S& s) {
        s.putf(12 + (W - 6) / 4, e.wstep(FC(0), SpanC<W>::owf, SpanC<W>::alpha, s.p, 0));
    }
};

template <int W>
struct Vwma {  // No-talib.py:17-19
    static constexpr u64 kC = lb(0) | lb(W), kV = lb(0) | lb(W);
    static constexpr u64 kRt = 0, kGc = 0;
    static constexpr Cols kOut = col1(24 + (W - 6) / 4);
    RollMean mvc, mv;
    __device__ void init() { mvc.init(); mv.init(); }
    template <class S> __device__ void step(S& s) {
        if (s.p >= W) {
            const double vq = s.V(W);
            mvc.remove(pinf(vq * s.C(W)));
            mv.remove(vq);
        }
        const double v0 = s.V(0);
        mvc.add(pinf(v0 * s.C(0)));
        mv.add(v0);
        s.put(24 + (W - 6) / 4, mvc.result(s, W, s.rn->VC) / mv.result(s, W, s.rn->V));
    }
    template <class S> __device__ void fstep(S& s) {
        const double vq = FV(W);
        mvc.fremove(vq * FC(W));
        mv.fremove(vq);
        mvc.fadd(FV(0) * FC(0));
        mv.fadd(FV(0));
        // a volume mean can round to 0 -> track
        s.put(24 + (W - 6) / 4, mvc.fresult_pos<W>(s.rn->VC) / mv.fresult_pos<W>(s.rn->V));
    }
    template <class S> __device__ void wstep(S& s) {
        const bool rm = s.p >= W;
        const int n = rm ? W : s.p + 1;
        const double vq = rm ? FV(W) : 0.0, cq = rm ? FC(W) : 0.0;
        const double v0 = FV(0);
        mvc.wstep(vq * cq, v0 * FC(0), n);
        mv.wstep(vq, v0, n);
        const double r = mvc.fresult_pos<W>(s.rn->VC) / mv.fresult_pos<W>(s.rn->V);
        s.put(24 + (W - 6) / 4, s.p >= W - 1 ? r : qnan());
    }
};

template <int W>
struct Bbands {  // No-talib.py:22-26
    static constexpr u64 kC = lb(0) | lb(W), kV = 0;
    static constexpr u64 kRt = 0, kGc = 0;
    static constexpr Cols kOut = col1(36 + 2 * ((W - 14) / 6)) | col1(37 + 2 * ((W - 14) / 6));
    RollMean m;
    RollVar v;
    __device__ void init() { m.init(); v.init(); }
    template <class S> __device__ void step(S& s) {
        if (s.p >= W) {
            const double xr = s.C(W);
            m.remove(xr);
            v.remove(s, xr);
        }
        double x = s.C(0);
        m.add(x);
        v.add(s, x);
        double ma = m.result(s, W, s.rn->C), sd = zsqrt(v.result(s, W, s.rn->C));
        const int col = 36 + 2 * ((W - 14) / 6);
        s.put(col, ma + (2 * sd));
        s.put(col + 1, ma - (2 * sd));
    }
    template <class S> __device__ void fstep(S& s) {
        const double xr = FC(W), x = FC(0);
        m.fremove(xr);
        v.fremove<W>(xr);
        m.fadd(x);
        v.fadd<W>(x);
        const double ma = m.fresult_pos<W>(s.rn->C), sd = zsqrt(v.fresult<W>(s.rn->C));
        const int col = 36 + 2 * ((W - 14) / 6);
        s.putf(col, ma + (2 * sd));
        s.putf(col + 1, ma - (2 * sd));
    }
    template <class S> __device__ void wstep(S& s) {
        const bool rm = s.p >= W;
        const double x = FC(0);
        m.wstep(rm ? FC(W) : 0.0, x, rm ? W : s.p + 1);
        if (rm) v.fremove<W>(FC(W));
        v.wadd(s, x, rm ? W : s.p + 1);
        const double ma = m.fresult_pos<W>(s.rn->C), sd = zsqrt(v.fresult<W>(s.rn->C));
        const bool full = s.p >= W - 1;
        const int col = 36 + 2 * ((W - 14) / 6);
        s.putf(col, full ? ma + (2 * sd) : qnan());
        s.putf(col + 1, full ? ma - (2 * sd) : qnan());
    }
};

template <int W>
struct MomAccelRocr {  // No-talib.py:35-44
    static constexpr u64 kC = lb(0) | lb(1) | lb(W) | lb(W + 1), kV = 0;
    static constexpr u64 kRt = 0, kGc = 0;
    static constexpr Cols kOut = col1(52 + (W - 14) / 6) | col1(60 + (W - 14) / 6) |
                                 col1(68 + (W - 14) / 6);
    __device__ void init() {}
    template <class S> __device__ void step(S& s) {
        const int k = (W - 14) / 6;
        double c = s.C(0);
        const double cw = s.C(W);
        double mom = c - cw, roc = c / cw - 1;
        double acc = mom - (s.C(1) - s.C(1 + W));
        mom = s.p >= W ? mom : qnan();
        roc = s.p >= W ? roc : qnan();
        acc = s.p >= W + 1 ? acc : qnan();
        s.put(52 + k, mom);
        s.put(60 + k, acc);
        s.put(68 + k, roc);
    }
    template <class S> __device__ void fstep(S& s) {
        const int k = (W - 14) / 6;
        const double c = FC(0), cw = FC(W);
        const double mom = c - cw;
        s.putf(52 + k, mom);
        s.putf(60 + k, mom - (FC(1) - FC(1 + W)));
        s.putf(68 + k, c / cw - 1);
    }
    template <class S> __device__ void wstep(S& s) {
        const int k = (W - 14) / 6;
        const double c = FC(0), cw = FC(W);
        const double mom = c - cw;
        s.putf(52 + k, s.p >= W ? mom : qnan());
        s.putf(60 + k, s.p >= W + 1 ? mom - (FC(1) - FC(1 + W)) : qnan());
        s.putf(68 + k, s.p >= W ? c / cw - 1 : qnan());
    }
};

template <int SLOW>
struct Macd {  // No-talib.py:47-50
    static constexpr u64 kC = lb(0), kV = 0;
    static constexpr u64 kRt = 0, kGc = 0;
    static constexpr Cols kOut = col1(76 + (SLOW - 18) / 6);
    Ewm fast, slow;
    __device__ void init() { fast.init(); slow.init(); }
    template <class S> __device__ void step(S& s) {
        double c = s.C(0);
        double f = fast.step(c, SpanC<12>::owf, SpanC<12>::alpha);
        double l = slow.step(c, SpanC<SLOW>::owf, SpanC<SLOW>::alpha);
        s.put(76 + (SLOW - 18) / 6, f - l);
    }
    template <class S> __device__ void fstep(S& s) {
        const double c = FC(0);
        const double f = fast.fstep(c, SpanC<12>::owf, SpanC<12>::alpha);
        const double l = slow.fstep(c, SpanC<SLOW>::owf, SpanC<SLOW>::alpha);
        s.putf(76 + (SLOW - 18) / 6, f - l);
    }
    template <class S> __device__ void wstep(S& s) {
        const double c = FC(0);
        const double f = fast.wstep(c, SpanC<12>::owf, SpanC<12>::alpha, s.p, 0);
        const double l = slow.wstep(c, SpanC<SLOW>::owf, SpanC<SLOW>::alpha, s.p, 0);
        s.putf(76 + (SLOW - 18) / 6, f - l);
    }
};

template <int I>
struct Rsi {  // No-talib.py:53-59
    static constexpr u64 kC = lb(0) | lb(1), kV = 0;
    static constexpr u64 kRt = 0, kGc = 0;
    static constexpr Cols kOut = col1(79 + (I - 8) / 6);
    Ewm up, dn;
    __device__ void init() { up.init(); dn.init(); }
    template <class S> __device__ void step(S& s) {
        double d = s.p >= 1 ? s.C(0) - s.C(1) : qnan();
        bool nan = (d != d);
        double u = (nan || d >= 0) ? d : 0.0;          // delta.clip(lower=0)
        double w = -((nan || d <= 0) ? d : 0.0);       // -delta.clip(upper=0)
        double eu = up.step(u, ComC<I - 1>::owf, ComC<I - 1>::alpha);
        double ed = dn.step(w, ComC<I - 1>::owf, ComC<I - 1>::alpha);
        double rs = eu / ed;
        s.put(79 + (I - 8) / 6, 100 - (100 / (1 + rs)));
    }
    template <class S> __device__ void fstep(S& s) {
        const double d = FC(0) - FC(1);
        const double u = d >= 0 ? d : 0.0;
        const double w = -(d <= 0 ? d : 0.0);
        const double eu = up.fstep(u, ComC<I - 1>::owf, ComC<I - 1>::alpha);
        const double ed = dn.fstep(w, ComC<I - 1>::owf, ComC<I - 1>::alpha);
        const double rs = eu / ed;
        s.put(79 + (I - 8) / 6, 100 - (100 / (1 + rs)));     // 0 / 0 on flat prices -> track
    }
    // the up / down moves are observed from p = 1 (day 0's diff is NaN: both ewms stay NaN)
    template <class S> __device__ void wstep(S& s) {
        const double d = FC(0) - FC(1);
        const double u = d >= 0 ? d : 0.0;
        const double w = -(d <= 0 ? d : 0.0);
        const double eu = up.wstep(u, ComC<I - 1>::owf, ComC<I - 1>::alpha, s.p, 1);
        const double ed = dn.wstep(w, ComC<I - 1>::owf, ComC<I - 1>::alpha, s.p, 1);
        const double rs = eu / ed;
        s.put(79 + (I - 8) / 6, 100 - (100 / (1 + rs)));
    }
};

struct PvtObvPsy {  // No-talib.py:62-69
    static constexpr u64 kC = lb(0) | lb(1) | lb(14) | lb(15), kV = lb(0);
    static constexpr u64 kRt = lb(0), kGc = 0;      // PVT's close.pct_change()
    static constexpr Cols kOut = col1(82) | col1(83) | col1(84);
    double pvt, obv;
    int ups;
    __device__ void init() { pvt = 0.0; obv = 0.0; ups = 0; }
    template <class S> __device__ void step(S& s) {
        const int p = s.p;
        double c = s.C(0), v = s.V(0);
        // PVT: nan-skipping cumsum of volume * pct_change (r0: NaN on observation 0)
        double term = v * s.ret(0);
        if (term == term) pvt = pvt + term;
        s.put(82, term == term ? pvt : qnan());
        // OBV: diff <= 0 (incl. equal closes) -> -volume, else (incl. NaN diff) +volume
        double d = p >= 1 ? c - s.C(1) : qnan();
        double o = v * ((d <= 0) ? -1.0 : 1.0);
        if (o == o) obv = obv + o;
        s.put(83, o == o ? obv : qnan());
        // PSY: rolling(14) count of up-days / 14 * 100 (0/1 sums are exact)
        ups += (p >= 1 && c > s.C(1)) ? 1 : 0;
        ups -= (p >= 15 && s.C(14) > s.C(15)) ? 1 : 0;
        s.put(84, p >= 13 ? s.div((double)ups, 14) * 100 : qnan());
    }
    template <class S> __device__ void fstep(S& s) {
        const double c = FC(0), v = FV(0), c1 = FC(1);
        pvt = pvt + v * s.template fret<0>();
        s.put(82, pvt);                                   // an earlier inf term persists -> track
        obv = obv + v * ((c - c1 <= 0) ? -1.0 : 1.0);
        s.put(83, obv);
        ups += (c > c1 ? 1 : 0) - (FC(14) > FC(15) ? 1 : 0);
        s.putf(84, divc<14>((double)ups) * 100);
    }
    template <class S> __device__ void wstep(S& s) {
        const int p = s.p;
        const double c = FC(0), v = FV(0), c1 = FC(1);
        const double pv = pvt + v * s.template fret<0>();
        pvt = p >= 1 ? pv : pvt;
        s.put(82, p >= 1 ? pvt : qnan());
        obv = obv + v * ((p >= 1 && c - c1 <= 0) ? -1.0 : 1.0);   // day 0: NaN diff -> +volume
        s.put(83, obv);
        ups += (p >= 1 && c > c1 ? 1 : 0) - (p >= 15 && FC(14) > FC(15) ? 1 : 0);
        s.putf(84, p >= 13 ? divc<14>((double)ups) * 100 : qnan());
    }
};

template <int W, int COL>
struct RetSd {  // sd_W of close.pct_change() (No-talib.py:72-74)
    static constexpr int kCol = COL;
    static constexpr u64 kC = 0, kV = 0, kRt = lb(0) | lb(W), kGc = 0;
    RollVar v;
    __device__ void init() { v.init(); }
    template <class S> __device__ double step(S& s) {
        if (s.p >= W) v.remove(s, pinf(s.ret(W)));
        v.add(s, pinf(s.ret(0)));
        double r = zsqrt(v.result(s, W, s.rn->R));
        s.put(COL, r);
        return r;
    }
    template <class S> __device__ double fstep(S& s) {
        v.fremove<W>(s.template fret<W>());
        v.fadd<W>(s.template fret<0>());
        const double r = zsqrt(v.fresult<W>(s.rn->R));
        s.putf(COL, r);
        return r;
    }
    // returns start at p = 1: the window holds min(p, W) of them, the first remove is at W + 1
    template <class S> __device__ double wstep(S& s) {
        if (s.p >= W + 1) v.fremove<W>(s.template fret<W>());
        if (s.p >= 1) v.wadd(s, s.template fret<0>(), s.p >= W ? W : s.p);
        const double r = s.p >= W ? zsqrt(v.fresult<W>(s.rn->R)) : qnan();
        s.putf(COL, r);
        return r;
    }
};

struct RetSd3 {
    RetSd<3, 85> a;
    static constexpr u64 kC = RetSd<3, 85>::kC, kV = 0, kRt = RetSd<3, 85>::kRt, kGc = 0;
    static constexpr Cols kOut = col1(85);
    __device__ void init() { a.init(); }
    template <class S> __device__ void step(S& s) { a.step(s); }
    template <class S> __device__ void fstep(S& s) { a.fstep(s); }
    template <class S> __device__ void wstep(S& s) { a.wstep(s); }
};

struct RetSd5x15 {  // sd_5, sd_15, sd5_15
    RetSd<5, 86> a;
    RetSd<15, 87> b;
    static constexpr u64 kC = RetSd<5, 86>::kC | RetSd<15, 87>::kC, kV = 0;
    static constexpr u64 kRt = RetSd<5, 86>::kRt | RetSd<15, 87>::kRt, kGc = 0;
    static constexpr Cols kOut = col1(86) | col1(87) | col1(88);
    __device__ void init() { a.init(); b.init(); }
    template <class S> __device__ void step(S& s) {
        double x = a.step(s), y = b.step(s);
        s.put(88, x / y);
    }
    template <class S> __device__ void fstep(S& s) {
        double x = a.fstep(s), y = b.fstep(s);
        s.put(88, x / y);
    }
    template <class S> __device__ void wstep(S& s) {
        double x = a.wstep(s), y = b.wstep(s);
        s.put(88, x / y);
    }
};

template <int W, int COL>
struct VolSd {  // volsd_W (No-talib.py:79-80)
    static constexpr int kCol = COL;
    static constexpr u64 kC = 0, kV = lb(0) | lb(W);
    static constexpr u64 kRt = 0, kGc = 0;
    RollVar v;
    __device__ void init() { v.init(); }
    template <class S> __device__ double step(S& s) {
        if (s.p >= W) v.remove(s, pinf(s.V(W)));
        v.add(s, pinf(s.V(0)));
        double r = zsqrt(v.result(s, W, s.rn->VP));
        s.put(COL, r);
        return r;
    }
    template <class S> __device__ double fstep(S& s) {
        v.fremove<W>(FV(W));
        v.fadd<W>(FV(0));
        const double r = zsqrt(v.fresult<W>(s.rn->VP));
        s.putf(COL, r);
        return r;
    }
    template <class S> __device__ double wstep(S& s) {
        if (s.p >= W) v.fremove<W>(FV(W));
        v.wadd(s, FV(0), s.p >= W ? W : s.p + 1);
        const double r = s.p >= W - 1 ? zsqrt(v.fresult<W>(s.rn->VP)) : qnan();
        s.putf(COL, r);
        return r;
    }
};

struct VolSd3 {
    VolSd<3, 89> a;
    static constexpr u64 kC = 0, kV = VolSd<3, 89>::kV;
    static constexpr u64 kRt = 0, kGc = 0;
    static constexpr Cols kOut = col1(89);
    __device__ void init() { a.init(); }
    template <class S> __device__ void step(S& s) { a.step(s); }
    template <class S> __device__ void fstep(S& s) { a.fstep(s); }
    template <class S> __device__ void wstep(S& s) { a.wstep(s); }
};

struct VolSd5x15 {
    VolSd<5, 90> a;
    VolSd<15, 91> b;
    static constexpr u64 kC = 0, kV = VolSd<5, 90>::kV | VolSd<15, 91>::kV;
    static constexpr u64 kRt = 0, kGc = 0;
    static constexpr Cols kOut = col1(90) | col1(91) | col1(92);
    __device__ void init() { a.init(); b.init(); }
    template <class S> __device__ void step(S& s) {
        double x = a.step(s), y = b.step(s);
        s.put(92, x / y);
    }
    template <class S> __device__ void fstep(S& s) {
        double x = a.fstep(s), y = b.fstep(s);
        s.put(92, x / y);
    }
    template <class S> __device__ void wstep(S& s) {
        double x = a.wstep(s), y = b.wstep(s);
        s.put(92, x / y);
    }
};

// sd5_15 / volsd5_15 split over two waves (PartT): the sd_5 wave writes its value of every present
// day into exchange slot SLOT's numerator (NUM), the sd_15 wave into its denominator, and the wave
// holding Comb<2> / Comb<3> stores x / y one chunk later -- the division RetSd5x15 / VolSd5x15
// make, on the same values, so columns 88 / 92 are bit-identical (and their NaN bits are the
// combiner's).  J = RetSd<W, COL> or VolSd<W, COL>; the sd column itself is stored as in the
// unsplit job.
template <class J, int SLOT, bool NUM>
struct XSd {
    static constexpr u64 kC = J::kC, kV = J::kV, kRt = J::kRt, kGc = J::kGc;
    static constexpr Cols kOut = col1(J::kCol);
    J a;
    template <class S> __device__ __forceinline__ static void xput(S& s, double v) {
        static_assert(S::kRG, "the split ratio needs the SmemRG exchange");
        LDS SmemRG* rg = (LDS SmemRG*)s.sm;
        if constexpr (NUM) rg->xnum[SLOT][s.par][s.sday][s.lane] = v;
        else rg->xden[SLOT][s.par][s.sday][s.lane] = v;
    }
    __device__ void init() { a.init(); }
    template <class S> __device__ void step(S& s) { xput(s, a.step(s)); }
    template <class S> __device__ void fstep(S& s) { xput(s, a.fstep(s)); }
    template <class S> __device__ void wstep(S& s) { xput(s, a.wstep(s)); }
};

// ret.rolling(W).corr(vol_change) (No-talib.py:85-87; pandas Rolling.corr on prep_binary'd
// inputs).  WITH_VC also emits the vol_change column.
template <int W, bool WITH_VC>
struct Corr {
    static constexpr u64 kC = 0, kV = 0, kRt = lb(0) | lb(W), kGc = lb(0) | lb(W);
    static constexpr Cols kOut = col1(94 + (W == 15 ? 1 : 0)) | (WITH_VC ? col1(93) : Cols{0, 0});
    RollMean mxy, mx, my;
    RollVar vx, vy;
    int cnt;
    __device__ void init() {
        mxy.init(); mx.init(); my.init(); vx.init(); vy.init();
        cnt = 0;
    }
    template <class S>
    __device__ __forceinline__ static void xy(S& s, int L, double& X, double& Y) {
        double r = s.ret(L), g = s.volchg(L);
        X = pinf(r + 0 * g);
        Y = pinf(g + 0 * r);
    }
    template <class S> __device__ void step(S& s) {
        double X, Y;
        if (s.p >= W) {
            xy(s, W, X, Y);
            mxy.remove(X * Y);
            mx.remove(X);
            my.remove(Y);
            vx.remove(s, X);
            vy.remove(s, Y);
            double t0 = X + Y;
            cnt -= (t0 == t0) ? 1 : 0;
        }
        xy(s, 0, X, Y);
        mxy.add(X * Y);
        mx.add(X);
        my.add(Y);
        vx.add(s, X);
        vy.add(s, Y);
        double t = X + Y;
        cnt += (t == t) ? 1 : 0;
        double c = (double)cnt;
        const double cf = cnt >= 1 ? s.div(c, cnt - 1) : -c;      // c / (c - 1)
        double num = (mxy.result(s, W, s.rn->XY) - mx.result(s, W, s.rn->X) * my.result(s, W, s.rn->Y)) * cf;
        double den = __builtin_sqrt(vx.result(s, W, s.rn->X) * vy.result(s, W, s.rn->Y));
        s.put(94 + (W == 15 ? 1 : 0), num / den);
        if (WITH_VC) s.put(93, s.volchg(0));
    }
    // clean: X = ret, Y = vol_change (finite), cnt = W; c / (c - 1) is the constant W / (W - 1)
    template <class S> __device__ void fstep(S& s) {
        const double Xr = s.template fret<W>(), Yr = s.template fvolchg<W>();
        const double X = s.template fret<0>(), Y = s.template fvolchg<0>();
        const double XYr = Xr * Yr, XY = X * Y;
        mxy.fremove(XYr);
        mx.fremove(Xr);
        my.fremove(Yr);
        vx.fremove<W>(Xr);
        vy.fremove<W>(Yr);
        mxy.fadd(XY);
        mx.fadd(X);
        my.fadd(Y);
        vx.fadd<W>(X);
        vy.fadd<W>(Y);
        mxy.fsigns(XY, XYr);
        mx.fsigns(X, Xr);
        my.fsigns(Y, Yr);
        constexpr double cf = (double)W / (double)(W - 1);
        const double num = (mxy.fresult<W>(s.rn->XY) - mx.fresult<W>(s.rn->X) * my.fresult<W>(s.rn->Y)) * cf;
        const double den = __builtin_sqrt(vx.fresult<W>(s.rn->X) * vy.fresult<W>(s.rn->Y));
        s.put(94 + (W == 15 ? 1 : 0), num / den);
        if (WITH_VC) s.putf(93, Y);
    }
    // the pair starts at p = 1 (day 0's returns are NaN): min(p, W) pairs in the window, the
    // first remove at W + 1; removes of 0 before it are exact no-ops on the Kahan means
    template <class S> __device__ void wstep(S& s) {
        const bool rm = s.p >= W + 1, ad = s.p >= 1;
        const int n = s.p >= W ? W : s.p;
        const double Xr = rm ? s.template fret<W>() : 0.0, Yr = rm ? s.template fvolchg<W>() : 0.0;
        const double X = ad ? s.template fret<0>() : 0.0, Y = ad ? s.template fvolchg<0>() : 0.0;
        const double XYr = Xr * Yr, XY = X * Y;
        mxy.wstep(XYr, XY, n);
        mx.wstep(Xr, X, n);
        my.wstep(Yr, Y, n);
        if (rm) {
            vx.fremove<W>(Xr);
            vy.fremove<W>(Yr);
        }
        if (ad) {
            vx.wadd(s, X, n);
            vy.wadd(s, Y, n);
        }
        mxy.fsigns(XY, XYr);
        mx.fsigns(X, Xr);
        my.fsigns(Y, Yr);
        cnt = n;
        constexpr double cf = (double)W / (double)(W - 1);
        const double num = (mxy.fresult<W>(s.rn->XY) - mx.fresult<W>(s.rn->X) * my.fresult<W>(s.rn->Y)) * cf;
        const double den = __builtin_sqrt(vx.fresult<W>(s.rn->X) * vy.fresult<W>(s.rn->Y));
        s.put(94 + (W == 15 ? 1 : 0), s.p >= W ? num / den : qnan());
        if (WITH_VC) s.putf(93, ad ? s.template fvolchg<0>() : qnan());
    }
};

// The rolling correlation split over two waves of one workgroup (PartS, small grids: the unsplit
// Corr is ~180 VALU per step, the longest dependency chain of the kernel).  CorrM keeps the three
// rolling means and the count -> the numerator (mean(XY) - mean(X) mean(Y)) * c / (c - 1); CorrV
// the two rolling variances -> the denominator sqrt(var(X) var(Y)).  Each writes its value of
// every present day into the workgroup's exchange (SmemRG xnum / xden [K][parity][day]); the
// wave holding Comb<K> forms num / den one chunk later (run_wave).  The same operations on the
// same states as Corr, so the column is bit-identical.  Days before the window is full get a
// NaN numerator (NaN / den = the NaN Corr stores there).  Needs RG (returns from the rings).
template <int W, bool WITH_VC>
struct CorrM {
    static constexpr int K = W == 15 ? 1 : 0;
    static constexpr u64 kC = 0, kV = 0, kRt = lb(0) | lb(W), kGc = lb(0) | lb(W);
    static constexpr Cols kOut = WITH_VC ? col1(93) : Cols{0, 0};
    RollMean mxy, mx, my;
    int cnt;
    __device__ void init() {
        mxy.init(); mx.init(); my.init();
        cnt = 0;
    }
    template <class S> __device__ __forceinline__ static void xput(S& s, double v) {
        static_assert(S::kRG, "the split correlation needs the SmemRG exchange");
        ((LDS SmemRG*)s.sm)->xnum[K][s.par][s.sday][s.lane] = v;
    }
    template <class S> __device__ void step(S& s) {
        double X, Y;
        if (s.p >= W) {
            Corr<W, false>::xy(s, W, X, Y);
            mxy.remove(X * Y);
            mx.remove(X);
            my.remove(Y);
            double t0 = X + Y;
            cnt -= (t0 == t0) ? 1 : 0;
        }
        Corr<W, false>::xy(s, 0, X, Y);
        mxy.add(X * Y);
        mx.add(X);
        my.add(Y);
        double t = X + Y;
        cnt += (t == t) ? 1 : 0;
        double c = (double)cnt;
        const double cf = cnt >= 1 ? s.div(c, cnt - 1) : -c;      // c / (c - 1)
        xput(s, (mxy.result(s, W, s.rn->XY) - mx.result(s, W, s.rn->X) * my.result(s, W, s.rn->Y)) * cf);
        if (WITH_VC) s.put(93, s.volchg(0));
    }
    template <class S> __device__ void fstep(S& s) {
        const double Xr = s.template fret<W>(), Yr = s.template fvolchg<W>();
        const double X = s.template fret<0>(), Y = s.template fvolchg<0>();
        const double XYr = Xr * Yr, XY = X * Y;
        mxy.fremove(XYr);
        mx.fremove(Xr);
        my.fremove(Yr);
        mxy.fadd(XY);
        mx.fadd(X);
        my.fadd(Y);
        mxy.fsigns(XY, XYr);
        mx.fsigns(X, Xr);
        my.fsigns(Y, Yr);
        constexpr double cf = (double)W / (double)(W - 1);
        xput(s, (mxy.fresult<W>(s.rn->XY) - mx.fresult<W>(s.rn->X) * my.fresult<W>(s.rn->Y)) * cf);
        if (WITH_VC) s.putf(93, Y);
    }
    template <class S> __device__ void wstep(S& s) {
        const bool rm = s.p >= W + 1, ad = s.p >= 1;
        const int n = s.p >= W ? W : s.p;
        const double Xr = rm ? s.template fret<W>() : 0.0, Yr = rm ? s.template fvolchg<W>() : 0.0;
        const double X = ad ? s.template fret<0>() : 0.0, Y = ad ? s.template fvolchg<0>() : 0.0;
        const double XYr = Xr * Yr, XY = X * Y;
        mxy.wstep(XYr, XY, n);
        mx.wstep(Xr, X, n);
        my.wstep(Yr, Y, n);
        mxy.fsigns(XY, XYr);
        mx.fsigns(X, Xr);
        my.fsigns(Y, Yr);
        cnt = n;
        constexpr double cf = (double)W / (double)(W - 1);
        const double num = (mxy.fresult<W>(s.rn->XY) - mx.fresult<W>(s.rn->X) * my.fresult<W>(s.rn->Y)) * cf;
        xput(s, s.p >= W ? num : qnan());
        if (WITH_VC) s.putf(93, ad ? s.template fvolchg<0>() : qnan());
    }
};

template <int W>
struct CorrV {
    static constexpr int K = W == 15 ? 1 : 0;
    static constexpr u64 kC = 0, kV = 0, kRt = lb(0) | lb(W), kGc = lb(0) | lb(W);
    static constexpr Cols kOut{0, 0};
    RollVar vx, vy;
    __device__ void init() { vx.init(); vy.init(); }
    template <class S> __device__ __forceinline__ static void xput(S& s, double v) {
        static_assert(S::kRG, "the split correlation needs the SmemRG exchange");
        ((LDS SmemRG*)s.sm)->xden[K][s.par][s.sday][s.lane] = v;
    }
    template <class S> __device__ void step(S& s) {
        double X, Y;
        if (s.p >= W) {
            Corr<W, false>::xy(s, W, X, Y);
            vx.remove(s, X);
            vy.remove(s, Y);
        }
        Corr<W, false>::xy(s, 0, X, Y);
        vx.add(s, X);
        vy.add(s, Y);
        xput(s, __builtin_sqrt(vx.result(s, W, s.rn->X) * vy.result(s, W, s.rn->Y)));
    }
    template <class S> __device__ void fstep(S& s) {
        const double Xr = s.template fret<W>(), Yr = s.template fvolchg<W>();
        const double X = s.template fret<0>(), Y = s.template fvolchg<0>();
        vx.fremove<W>(Xr);
        vy.fremove<W>(Yr);
        vx.fadd<W>(X);
        vy.fadd<W>(Y);
        xput(s, __builtin_sqrt(vx.fresult<W>(s.rn->X) * vy.fresult<W>(s.rn->Y)));
    }
    template <class S> __device__ void wstep(S& s) {
        const bool rm = s.p >= W + 1, ad = s.p >= 1;
        const int n = s.p >= W ? W : s.p;
        if (rm) {
            vx.fremove<W>(s.template fret<W>());
            vy.fremove<W>(s.template fvolchg<W>());
        }
        if (ad) {
            vx.wadd(s, s.template fret<0>(), n);
            vy.wadd(s, s.template fvolchg<0>(), n);
        }
        xput(s, __builtin_sqrt(vx.fresult<W>(s.rn->X) * vy.fresult<W>(s.rn->Y)));
    }
};

// Marks the wave that combines split column K (kinds: see kCombs -- num / den of the previous
// chunk, its column stores and NaN bits; run_wave).  No per-day work.
template <int K>
struct Comb {
    static constexpr u64 kC = 0, kV = 0, kRt = 0, kGc = 0;
    static constexpr Cols kOut{0, 0};
    __device__ void init() {}
    template <class S> __device__ void step(S&) {}
    template <class S> __device__ void fstep(S&) {}
    template <class S> __device__ void wstep(S&) {}
};
template <class T> struct Comb_of { static constexpr unsigned value = 0; };
template <int K> struct Comb_of<Comb<K>> { static constexpr unsigned value = 1u << K; };

// ---- job packs ------------------------------------------------------------------------------
// Series flags: which per-step inputs / runs a pack reads.
enum : unsigned {
    kSerC = 1, kSerV = 2, kSerVP = 4, kSerVC = 8, kSerR = 16, kSerXY = 32,
};
template <class T> struct Ser { static constexpr unsigned value = 0; };
template <int W> struct Ser<Sma<W>> { static constexpr unsigned value = kSerC; };
template <int W> struct Ser<Bbands<W>> { static constexpr unsigned value = kSerC; };
template <int W> struct Ser<Vwma<W>> { static constexpr unsigned value = kSerV | kSerVC; };
template <> struct Ser<RetSd3> { static constexpr unsigned value = kSerR; };
template <> struct Ser<RetSd5x15> { static constexpr unsigned value = kSerR; };
template <> struct Ser<VolSd3> { static constexpr unsigned value = kSerVP; };
template <> struct Ser<VolSd5x15> { static constexpr unsigned value = kSerVP; };
template <int W, bool V> struct Ser<Corr<W, V>> { static constexpr unsigned value = kSerXY; };
template <int W, bool V> struct Ser<CorrM<W, V>> { static constexpr unsigned value = kSerXY; };
template <int W> struct Ser<CorrV<W>> { static constexpr unsigned value = kSerXY; };
template <int W, int C, int SL, bool N> struct Ser<XSd<RetSd<W, C>, SL, N>> {
    static constexpr unsigned value = kSerR;
};
template <int W, int C, int SL, bool N> struct Ser<XSd<VolSd<W, C>, SL, N>> {
    static constexpr unsigned value = kSerVP;
};

template <class... J>
struct Pack;
template <>
struct Pack<> {
    static constexpr unsigned kSer = 0, kComb = 0;
    static constexpr u64 kC = 0, kV = 0;
    static constexpr u64 kRt = 0, kGc = 0;
    static constexpr Cols kOut{0, 0};
    __device__ void init() {}
    template <class S> __device__ void step(S&) {}
    template <class S> __device__ void fstep(S&) {}
    template <class S> __device__ void wstep(S&) {}
};
template <class H, class... R>
struct Pack<H, R...> {
    static constexpr unsigned kSer = Ser<H>::value | Pack<R...>::kSer;
    // the lookbacks the jobs' clean / warm steps read
    static constexpr u64 kC = H::kC | Pack<R...>::kC, kV = H::kV | Pack<R...>::kV;
    static constexpr u64 kRt = H::kRt | Pack<R...>::kRt, kGc = H::kGc | Pack<R...>::kGc;
    // the split correlations this wave combines (bit k: corr k, see Comb)
    static constexpr unsigned kComb = Comb_of<H>::value | Pack<R...>::kComb;
    static constexpr Cols kOut = H::kOut | Pack<R...>::kOut;
    H h;
    Pack<R...> r;
    __device__ void init() { h.init(); r.init(); }
    // the general step (cold) runs its jobs one after the other: interleaving them would raise
    // the register pressure of the whole scan
    template <class S> __device__ void step(S& s) {
        h.step(s);
        __builtin_amdgcn_sched_barrier(0);
        r.step(s);
    }
    template <class S> __device__ void fstep(S& s) {
        h.fstep(s);     // no scheduling barrier: the compiler interleaves the jobs' independent
        r.fstep(s);     // chains (12.55 -> 12.32 ms at config C, bit-identical)
    }
    template <class S> __device__ void wstep(S& s) {
        h.wstep(s);
        __builtin_amdgcn_sched_barrier(0);
        r.wstep(s);
    }
};

// ---- partitions ----------------------------------------------------------------------------
// PartC (large grids, config C): the 15 job sets of one block, 3 item types of 5 job sets.
// Round 4: per type three light sets (the two rolling correlations alone, ...) at wave positions
// 0, 2, 4 -- the SIMDs that carry three job waves of a paired workgroup -- and two heavy ones
// (6-7 moving sums / bands) at positions 1, 3, the SIMDs the loaders share.  Config C: the same
// time as the round-3 partition (10.3-10.7 ms, the kernel is bound by its write stream there);
// at 1,250 assets, where each set runs alone on its SIMD (the 15-way split), 4.06 vs 4.30-4.54 ms
// -- the correlations no longer share a wave (tools/archive/gpu_r4i.sh, profiles/r4_i_partition_ab.txt).
// A variant that moved one moving sum from each heavy set to a light one ran slower at both
// sizes (11.0 / 4.7 ms).  The heavy sets' fast steps keep <= 8 scratch accesses (slab entry
// reloads; the day loop's chains have none).
struct PartC {
    static constexpr int kSets = 15;
    static constexpr bool kRG = false;
    static constexpr int kCombs = 0;
    template <int K> struct Set;
};
#ifdef AFM_FP_CENSUS_W0     // instruction census of one job alone (tools/job_census.sh)
template <> struct PartC::Set<0> { using type = Pack<AFM_FP_CENSUS_W0>; };
#else
template <> struct PartC::Set<0> { using type = Pack<Corr<5, true>>; };
#endif
template <> struct PartC::Set<1> { using type = Pack<Bbands<32>, Vwma<30>, MomAccelRocr<32>, Ema<30>, Ema<6>, Sma<30>, Sma<18>>; };
template <> struct PartC::Set<2> { using type = Pack<Bbands<14>, Vwma<14>, Ema<14>>; };
template <> struct PartC::Set<3> { using type = Pack<Bbands<38>, Vwma<38>, MomAccelRocr<38>, Ema<38>, Ema<10>, Sma<38>, Sma<22>>; };
template <> struct PartC::Set<4> { using type = Pack<Rsi<20>, Vwma<22>, MomAccelRocr<14>, Sma<14>, Macd<18>>; };
template <> struct PartC::Set<5> { using type = Pack<Corr<15, false>>; };
template <> struct PartC::Set<6> { using type = Pack<Bbands<44>, Vwma<42>, MomAccelRocr<44>, Ema<42>, Ema<22>, Sma<42>, Sma<26>>; };
template <> struct PartC::Set<7> { using type = Pack<Bbands<20>, Vwma<18>, Ema<18>>; };
template <> struct PartC::Set<8> { using type = Pack<Bbands<50>, Vwma<46>, MomAccelRocr<50>, Ema<46>, Ema<50>, Sma<46>, Sma<34>>; };
template <> struct PartC::Set<9> { using type = Pack<RetSd5x15, VolSd3, Sma<6>>; };
template <> struct PartC::Set<10> { using type = Pack<VolSd5x15, Rsi<8>>; };
template <> struct PartC::Set<11> { using type = Pack<Bbands<56>, Vwma<50>, Vwma<34>, MomAccelRocr<56>, Sma<50>>; };
template <> struct PartC::Set<12> { using type = Pack<PvtObvPsy, RetSd3, Rsi<14>, Sma<10>>; };
template <> struct PartC::Set<13> { using type = Pack<Vwma<6>, Vwma<10>, MomAccelRocr<20>, MomAccelRocr<26>, Ema<34>, Macd<24>, Macd<30>>; };
template <> struct PartC::Set<14> { using type = Pack<Bbands<26>, Vwma<26>, Ema<26>>; };

// PartS (small grids: a multi-GPU shard, configs B / D): 30 job sets of ~1-3 recurrences each,
// so that at a few dozen 64-asset blocks the longest per-wave dependency chain -- what bounds the
// kernel there (a lone wave per SIMD issues its own stream, ~260 + 5 x VALU cycles
// per day) -- is about half of PartC's.  The rolling correlations are split over two waves
// (CorrM / CorrV), the returns and volume changes come from the loader's rings (RG), and a
// workgroup holds J = 3, 5, 6 or 10 consecutive sets + a loader (140 KB of LDS: one per CU,
// the grid <= the CU count).  Each correlation's two halves and its combiner (on the CorrV wave)
// are sets 0-1 / 3-4, in one workgroup for every J.
struct PartS {
    static constexpr int kSets = 30;
    static constexpr bool kRG = true;
    static constexpr int kCombs = 2;                  // corr_5, corr_15
    template <int K> struct Set;
};
template <> struct PartS::Set<0> { using type = Pack<CorrM<5, true>, Ema<6>>; };
template <> struct PartS::Set<1> { using type = Pack<CorrV<5>, Comb<0>>; };
template <> struct PartS::Set<2> { using type = Pack<Bbands<14>, Ema<10>>; };
template <> struct PartS::Set<3> { using type = Pack<CorrM<15, false>, Ema<14>>; };
template <> struct PartS::Set<4> { using type = Pack<CorrV<15>, Comb<1>>; };
template <> struct PartS::Set<5> { using type = Pack<Bbands<20>, Ema<18>>; };
template <> struct PartS::Set<6> { using type = Pack<Bbands<26>, Sma<6>>; };
template <> struct PartS::Set<7> { using type = Pack<Bbands<32>, Sma<10>>; };
template <> struct PartS::Set<8> { using type = Pack<Bbands<38>, Sma<14>>; };
template <> struct PartS::Set<9> { using type = Pack<Bbands<44>, Sma<18>>; };
template <> struct PartS::Set<10> { using type = Pack<Bbands<50>, Sma<22>>; };
template <> struct PartS::Set<11> { using type = Pack<Bbands<56>, Sma<26>>; };
template <> struct PartS::Set<12> { using type = Pack<Vwma<6>, MomAccelRocr<14>>; };
template <> struct PartS::Set<13> { using type = Pack<Vwma<10>, MomAccelRocr<20>>; };
template <> struct PartS::Set<14> { using type = Pack<Vwma<14>, MomAccelRocr<26>>; };
template <> struct PartS::Set<15> { using type = Pack<Vwma<18>, MomAccelRocr<32>>; };
template <> struct PartS::Set<16> { using type = Pack<Vwma<22>, MomAccelRocr<38>>; };
template <> struct PartS::Set<17> { using type = Pack<Vwma<26>, MomAccelRocr<44>>; };
template <> struct PartS::Set<18> { using type = Pack<Vwma<30>, MomAccelRocr<50>>; };
template <> struct PartS::Set<19> { using type = Pack<Vwma<34>, MomAccelRocr<56>>; };
template <> struct PartS::Set<20> { using type = Pack<Vwma<38>, Sma<30>, Ema<30>>; };
template <> struct PartS::Set<21> { using type = Pack<Vwma<42>, Sma<34>, Ema<34>>; };
template <> struct PartS::Set<22> { using type = Pack<Vwma<46>, Sma<38>, Ema<38>>; };
template <> struct PartS::Set<23> { using type = Pack<Vwma<50>, Sma<42>, Ema<42>>; };
template <> struct PartS::Set<24> { using type = Pack<RetSd5x15>; };
template <> struct PartS::Set<25> { using type = Pack<VolSd5x15>; };
template <> struct PartS::Set<26> { using type = Pack<Rsi<8>, RetSd3, Ema<22>>; };
template <> struct PartS::Set<27> { using type = Pack<Rsi<14>, VolSd3, Ema<26>>; };
template <> struct PartS::Set<28> { using type = Pack<Rsi<20>, PvtObvPsy>; };
template <> struct PartS::Set<29> { using type = Pack<Macd<18>, Macd<24>, Macd<30>, Ema<46>, Ema<50>, Sma<46>, Sma<50>>; };

// PartT (26-42 blocks: the N = 4 shard; round 5): 60 job sets of ONE recurrence family each (a few
// pairs of light ones), 10 job waves + a loader per 140-KB workgroup (6 per block).  Besides the
// correlations, sd5_15 and volsd5_15 are split too (XSd: the sd_5 and sd_15 waves feed exchange
// slots 0 / 1 of their workgroup, Comb<2> / Comb<3> divide).  Sets 0-4 (the correlations and
// their combiners) and 30-34 (the sd ratios) lie inside one workgroup for J = 5, 6 and 10, and
// each of those workgroups uses exchange slots 0 and 1 once.  Measured at 2,500 assets: 3.27 vs
// PartS's 3.63 ms; at 1,250 it loses to PartS J = 3 (a small-grid job wave's cost is its per-day
// fixed chain, not its jobs: profiles/r5_rt_partitions.txt), so only J = 10 is built.
struct PartT {
    static constexpr int kSets = 60;
    static constexpr bool kRG = true;
    static constexpr int kCombs = 4;                  // corr_5, corr_15, sd5_15, volsd5_15
    template <int K> struct Set;
};
template <> struct PartT::Set<0> { using type = Pack<CorrM<5, true>>; };
template <> struct PartT::Set<1> { using type = Pack<CorrV<5>>; };
template <> struct PartT::Set<2> { using type = Pack<CorrM<15, false>>; };
template <> struct PartT::Set<3> { using type = Pack<CorrV<15>>; };
template <> struct PartT::Set<4> { using type = Pack<Comb<0>, Comb<1>, Ema<6>>; };
template <> struct PartT::Set<5> { using type = Pack<Bbands<14>>; };
template <> struct PartT::Set<6> { using type = Pack<Vwma<6>>; };
template <> struct PartT::Set<7> { using type = Pack<Bbands<20>>; };
template <> struct PartT::Set<8> { using type = Pack<Vwma<10>>; };
template <> struct PartT::Set<9> { using type = Pack<Sma<6>>; };
template <> struct PartT::Set<10> { using type = Pack<Bbands<26>>; };
template <> struct PartT::Set<11> { using type = Pack<Vwma<14>>; };
template <> struct PartT::Set<12> { using type = Pack<Bbands<32>>; };
template <> struct PartT::Set<13> { using type = Pack<Vwma<18>>; };
template <> struct PartT::Set<14> { using type = Pack<Sma<10>>; };
template <> struct PartT::Set<15> { using type = Pack<Bbands<38>>; };
template <> struct PartT::Set<16> { using type = Pack<Vwma<22>>; };
template <> struct PartT::Set<17> { using type = Pack<Bbands<44>>; };
template <> struct PartT::Set<18> { using type = Pack<Vwma<26>>; };
template <> struct PartT::Set<19> { using type = Pack<Sma<14>>; };
template <> struct PartT::Set<20> { using type = Pack<Bbands<50>>; };
template <> struct PartT::Set<21> { using type = Pack<Vwma<30>>; };
template <> struct PartT::Set<22> { using type = Pack<Bbands<56>>; };
template <> struct PartT::Set<23> { using type = Pack<Vwma<34>>; };
template <> struct PartT::Set<24> { using type = Pack<Sma<18>>; };
template <> struct PartT::Set<25> { using type = Pack<Rsi<8>>; };
template <> struct PartT::Set<26> { using type = Pack<Vwma<38>>; };
template <> struct PartT::Set<27> { using type = Pack<Rsi<14>>; };
template <> struct PartT::Set<28> { using type = Pack<Vwma<42>>; };
template <> struct PartT::Set<29> { using type = Pack<Sma<22>>; };
template <> struct PartT::Set<30> { using type = Pack<XSd<RetSd<5, 86>, 0, true>>; };
template <> struct PartT::Set<31> { using type = Pack<XSd<RetSd<15, 87>, 0, false>>; };
template <> struct PartT::Set<32> { using type = Pack<XSd<VolSd<5, 90>, 1, true>>; };
template <> struct PartT::Set<33> { using type = Pack<XSd<VolSd<15, 91>, 1, false>>; };
template <> struct PartT::Set<34> { using type = Pack<Comb<2>, Comb<3>, Ema<10>>; };
template <> struct PartT::Set<35> { using type = Pack<Rsi<20>>; };
template <> struct PartT::Set<36> { using type = Pack<Vwma<46>>; };
template <> struct PartT::Set<37> { using type = Pack<PvtObvPsy>; };
template <> struct PartT::Set<38> { using type = Pack<Vwma<50>>; };
template <> struct PartT::Set<39> { using type = Pack<Sma<26>>; };
template <> struct PartT::Set<40> { using type = Pack<MomAccelRocr<14>>; };
template <> struct PartT::Set<41> { using type = Pack<RetSd3, Ema<14>>; };
template <> struct PartT::Set<42> { using type = Pack<MomAccelRocr<20>>; };
template <> struct PartT::Set<43> { using type = Pack<VolSd3, Ema<18>>; };
template <> struct PartT::Set<44> { using type = Pack<Sma<30>>; };
template <> struct PartT::Set<45> { using type = Pack<MomAccelRocr<26>>; };
template <> struct PartT::Set<46> { using type = Pack<Macd<18>, Ema<22>>; };
template <> struct PartT::Set<47> { using type = Pack<MomAccelRocr<32>>; };
template <> struct PartT::Set<48> { using type = Pack<Macd<24>, Ema<26>>; };
template <> struct PartT::Set<49> { using type = Pack<Sma<34>>; };
template <> struct PartT::Set<50> { using type = Pack<MomAccelRocr<38>>; };
template <> struct PartT::Set<51> { using type = Pack<Macd<30>, Ema<30>>; };
template <> struct PartT::Set<52> { using type = Pack<MomAccelRocr<44>>; };
template <> struct PartT::Set<53> { using type = Pack<Sma<38>, Ema<34>>; };
template <> struct PartT::Set<54> { using type = Pack<Sma<42>, Ema<38>>; };
template <> struct PartT::Set<55> { using type = Pack<MomAccelRocr<50>>; };
template <> struct PartT::Set<56> { using type = Pack<Sma<46>, Ema<42>>; };
template <> struct PartT::Set<57> { using type = Pack<MomAccelRocr<56>>; };
template <> struct PartT::Set<58> { using type = Pack<Sma<50>, Ema<46>>; };
template <> struct PartT::Set<59> { using type = Pack<Ema<50>>; };

// mask partials of a partition: one per job set + one per split correlation's combiner
template <class Part> constexpr int nparts() { return Part::kSets + Part::kCombs; }

// The loader wave: global -> ring, one chunk ahead.  Executes the same barrier sequence as the
// job waves (one per chunk).  It also publishes, per lane and chunk, whether every present day of
// the chunk is clean (kClean).  RG: it also computes each observation's close.pct_change() and
// volume.pct_change() (the same IEEE expressions the job waves would: x / x_prev - 1, NaN for an
// asset's first observation) into the SmemRG rings, index = observation mod kRingR.
// State words (slab carry): the rings, pmod, run, cnt; RG: + the r / g rings, obs mod kRingR.
template <bool RG>
constexpr int loader_state_words() { return 2 * kRing + 3 + (RG ? 2 * kRingR + 1 : 0); }
template <bool RG>
__device__ __forceinline__ void load_wave(const Args& a, LDS Smem* smp, int lane, int64_t block,
                                          GLB double* st) {
    LDS Smem& sm = *smp;
    LDS SmemRG* rg = (LDS SmemRG*)smp;
    const int64_t asset = block * kLanes + lane_asset(lane);
    const int c0 = a.c0, nch = a.c1;
    // kPre chunks of loads in flight (round 5: with one, the loader's load latency bounded every
    // small-grid workgroup at ~4.9 Mcycles -- ~970 cycles per day -- whatever its job sets,
    // profiles/r5_s_wave_profiles.txt)
    constexpr int kPre = 3;
    double pc[kPre][kChunk], pv[kPre][kChunk];
    u64 pw[kPre];                                   // each staged chunk's presence word
    int pmod = 0;                                   // observations before the staged chunk, mod kRing
    int run = 0;                                    // consecutive in-range observations (cap kClean)
    int cnt = 0;                                    // observations (capped at kClean)
    int p32 = 0;                                    // RG: observations mod kRingR
    if (st && a.load_state) {                       // the ring and counters of the previous slab
        for (int q = 0; q < kRing; ++q) {
            sm.c[q][lane] = st[(2 * q) * kLanes + lane];
            sm.v[q][lane] = st[(2 * q + 1) * kLanes + lane];
        }
        pmod = (int)st[(2 * kRing) * kLanes + lane];
        run = (int)st[(2 * kRing + 1) * kLanes + lane];
        cnt = (int)st[(2 * kRing + 2) * kLanes + lane];
        if constexpr (RG) {
            for (int q = 0; q < kRingR; ++q) {
                rg->r[q][lane] = st[(2 * kRing + 3 + 2 * q) * kLanes + lane];
                rg->g[q][lane] = st[(2 * kRing + 4 + 2 * q) * kLanes + lane];
            }
            p32 = (int)st[(2 * kRing + 3 + 2 * kRingR) * kLanes + lane];
        }
    }
    // RG: the previous observation's close / volume (the ring's newest entry)
    double cprev = 0.0, vprev = 0.0;
    if constexpr (RG) {
        const int q = pmod == 0 ? kRing - 1 : pmod - 1;
        cprev = sm.c[q][lane];
        vprev = sm.v[q][lane];
    }
    // Every load is issued on every path -- a chunk past the slab re-reads the slab's last chunk,
    // a date past t1 re-reads row t1 - 1, values that are never staged -- and consumed only when
    // staged: a load consumed where it is issued, or issued under a condition, makes the compiler
    // wait for the whole prefetch there ("compiler waits")
    auto load = [&](int ch, double (&xc)[kChunk], double (&xv)[kChunk], u64& w) {
        const int chc = ch < nch ? ch : nch - 1;
        w = a.vbits[(int64_t)((chc * kChunk) >> 6) * a.lda + asset];
#pragma unroll
        for (int j = 0; j < kChunk; ++j) {
            const int64_t t = (int64_t)chc * kChunk + j;
            const int64_t tc = t < a.t1 ? t : a.t1 - 1;
            xc[j] = a.close[tc * a.lda + asset];
            xv[j] = a.volume[tc * a.lda + asset];
        }
    };
    // registers (chunk ch) -> ring + cbyte (dates past t1 stage 0: never present there, as the
    // slabs end on a 64-date word or at T)
    auto stage = [&](int ch, const double (&xc)[kChunk], const double (&xv)[kChunk], u64 w) {
        const int sh = (ch * kChunk) & 63;
        const u64 cb = (w >> sh) & 0xffull;
        int q = pmod;
        bool ok = true, warm = true;
#pragma unroll
        for (int j = 0; j < kChunk; ++j) {
            if ((cb >> j) & 1ull) {
                const bool in = (int64_t)ch * kChunk + j < a.t1;
                const double cj = in ? xc[j] : 0.0, vj = in ? xv[j] : 0.0;
                sm.c[q][lane] = cj;
                sm.v[q][lane] = vj;
                if constexpr (RG) {
                    const double r = cj / cprev - 1, g = vj / vprev - 1;
                    rg->r[p32][lane] = cnt > 0 ? r : qnan();
                    rg->g[p32][lane] = cnt > 0 ? g : qnan();
                    cprev = cj;
                    vprev = vj;
                    p32 = (p32 + 1) & (kRingR - 1);
                }
                q = q + 1 == kRing ? 0 : q + 1;
                const bool good = cj > kLo && cj < kHi && vj > kLo && vj < kHi;
                run = good ? (run < kClean ? run + 1 : kClean) : 0;
                cnt = cnt < kClean ? cnt + 1 : kClean;
                ok = ok && run >= kClean;
                warm = warm && (run >= kClean || run == cnt);   // every observation so far good
            }
        }
        pmod = q;
        sm.cbyte[ch & 1][lane] = (int)cb;
        sm.okbyte[ch & 1][lane] = !a.fast ? 0 : ok ? 2 : warm ? 1 : 0;
    };
    static_assert(kPre == 3, "the loop below is unrolled for three buffers");
    load(c0, pc[0], pv[0], pw[0]);
    load(c0 + 1, pc[1], pv[1], pw[1]);
    load(c0 + 2, pc[2], pv[2], pw[2]);
    stage(c0, pc[0], pv[0], pw[0]);
    lds_barrier();                                  // chunk c0 staged
    // iteration ch = c0 + i: stage chunk ch + 1 (buffer (i + 1) % 3), then load chunk ch + 3 into
    // buffer i % 3 (chunk ch's, staged one iteration ago); one barrier per chunk, as the job waves
    auto iter = [&](int ch, auto bc) {
        constexpr int b = decltype(bc)::value, bn = (b + 1) % kPre;
        if (ch + 1 < nch) stage(ch + 1, pc[bn], pv[bn], pw[bn]);
        load(ch + 3, pc[b], pv[b], pw[b]);
        lds_barrier();
    };
    for (int ch = c0; ch < nch; ch += kPre) {
        iter(ch, std::integral_constant<int, 0>{});
        if (ch + 1 >= nch) break;
        iter(ch + 1, std::integral_constant<int, 1>{});
        if (ch + 2 >= nch) break;
        iter(ch + 2, std::integral_constant<int, 2>{});
    }
    if (st) {                                       // for the next slab (after the last barrier:
        for (int q = 0; q < kRing; ++q) {           // no job wave reads the ring any more)
            st[(2 * q) * kLanes + lane] = sm.c[q][lane];
            st[(2 * q + 1) * kLanes + lane] = sm.v[q][lane];
        }
        st[(2 * kRing) * kLanes + lane] = (double)pmod;
        st[(2 * kRing + 1) * kLanes + lane] = (double)run;
        st[(2 * kRing + 2) * kLanes + lane] = (double)cnt;
        if constexpr (RG) {
            for (int q = 0; q < kRingR; ++q) {
                st[(2 * kRing + 3 + 2 * q) * kLanes + lane] = rg->r[q][lane];
                st[(2 * kRing + 4 + 2 * q) * kLanes + lane] = rg->g[q][lane];
            }
            st[(2 * kRing + 3 + 2 * kRingR) * kLanes + lane] = (double)p32;
        }
    }
}

// A wave with no item (odd item count in the paired launch): the loader's barrier sequence.
__device__ __forceinline__ void idle_wave(const Args& a) {
    const int nch = a.c1;
    lds_barrier();
    for (int ch = a.c0; ch < nch; ++ch) lds_barrier();
}

// A job wave's complete state between two time slabs (stored lane-interleaved, 8-B words)
template <class P>
struct JobState {
    P jobs;
    Runs rn;
    int pos, pmod;
};
template <class P>
__device__ __forceinline__ void state_io(GLB double* st, JobState<P>& js, int lane, bool save) {
    constexpr int n = (int)((sizeof(JobState<P>) + 7) / 8);
    double w[n];
    if (save) {
        __builtin_memcpy(w, &js, sizeof(JobState<P>));
        for (int i = 0; i < n; ++i) st[i * kLanes + lane] = w[i];
    } else {
        for (int i = 0; i < n; ++i) w[i] = st[i * kLanes + lane];
        __builtin_memcpy(&js, w, sizeof(JobState<P>));
    }
}

template <class P, bool RG>
__device__ __forceinline__ void run_wave(const Args& a, LDS Smem* smp, int type, int wave, int lane,
                                      int64_t block, GLB double* stp) {
    LDS Smem& sm = *smp;
    // this lane's byte offset inside a date row: every output / mask store is an SGPR row base
    // plus this offset (no 64-bit per-lane address kept live through the scan)
    const uint32_t voff = (uint32_t)((block * kLanes + lane_asset(lane)) * 8);
    const int c0 = a.c0, nch = a.c1;
    const int64_t w0 = ((int64_t)c0 * kChunk) >> 6;                     // the slab's first word
    constexpr unsigned S = P::kSer;
    // the return / volume-change lookbacks: the jobs' own, plus lookback 0 for the runs of the
    // returns (R) and of the correlation pair (XY)
    constexpr u64 RT = P::kRt | ((S & (kSerR | kSerXY)) ? lb(0) : 0ull);
    constexpr u64 GC = P::kGc | ((S & kSerXY) ? lb(0) : 0ull);
    // clean / warm steps: the pack's lookbacks; without the rings (RG) a return at lookback L is
    // divided from close L and L + 1 (volume likewise)
    constexpr u64 CM = P::kC | lb(0) | (RG ? 0ull : (RT | (RT << 1)));
    constexpr u64 VM = P::kV | lb(0) | (RG ? 0ull : (GC | (GC << 1)));
    constexpr unsigned KC = P::kComb;
    static_assert(RG || KC == 0, "the correlation combiner needs the SmemRG exchange");
    P jobs;
    jobs.init();
    Runs rn;
    rn.C.init(); rn.V.init(); rn.VP.init(); rn.VC.init();
    rn.R.init(); rn.X.init(); rn.Y.init(); rn.XY.init();
    int pos = 0, pmod = 0;      // observations of this lane before the current chunk (and mod kRing)
    if (stp && a.load_state) {
        JobState<P> js;
        state_io(stp, js, lane, false);
        jobs = js.jobs;
        rn = js.rn;
        pos = js.pos;
        pmod = js.pmod;
    }
    u64 nb = 0ull, fb = 0ull;   // this wave's NaN / non-finite bits of the current 64-day word
    u64 cnb[kCombs] = {0ull, 0ull, 0ull, 0ull}, cfb[kCombs] = {0ull, 0ull, 0ull, 0ull};   // the combiner's
    lds_barrier();              // chunk 0 staged
#ifdef AFM_FP_PROFILE
    const long long tstart = __builtin_readcyclecounter();
    const long long treal = (long long)__builtin_amdgcn_s_memrealtime();   // 100 MHz, chip-wide
    long long twait = 0;
#endif

    FastStep<RG, CM, VM, RT, GC> st;
    st.sm = smp;
    st.rn = &rn;
    st.plane = a.plane;
    st.voff = voff;
    st.poff = (uint32_t)((block * kLanes + 2 * (lane & 31)) * 8);
    st.hmask = lane >= 32 ? -1 : 0;
    st.lane = lane;
    using FS = FastStep<RG, CM, VM, RT, GC>;
    // one clean day of step object x (its ring offsets set): gather, the per-day values and
    // runs, the jobs' fast steps, the day's NaN bits
    auto fast_day = [&](FS& x, int s, unsigned& n8, unsigned& f8) {
        x.sday = s;
        x.anynan = false;
        x.anybad = false;
        const double c0 = x.template c<0>(), v0 = x.template v<0>();
        if constexpr ((RT & 1ull) != 0) {
            if constexpr (RG) x.r0 = x.rr[0];
            else x.r0 = c0 / x.template c<1>() - 1;
        }
        if constexpr ((GC & 1ull) != 0) {
            if constexpr (RG) x.g0 = x.gg[0];
            else x.g0 = v0 / x.template v<1>() - 1;
        }
        if (S & kSerC) rn.C.fupd(c0);
        if (S & kSerV) rn.V.fupd(v0);
        if (S & kSerVP) rn.VP.fupd(v0);
        if (S & kSerVC) rn.VC.fupd(v0 * c0);
        if (S & kSerR) rn.R.fupd(x.r0);
        if (S & kSerXY) {
            rn.X.fupd(x.r0);
            rn.Y.fupd(x.g0);
            rn.XY.fupd(x.r0 * x.g0);
        }
        jobs.fstep(x);
        n8 |= x.anynan ? 1u << s : 0u;
        f8 |= x.anybad ? 1u << s : 0u;
    };
    // per present day: the ring offsets of observation p (pm = p mod kRing)
    auto set_day = [&](FS& x, int p, int pm) {
        x.p = p;
        x.pmoff = (uint32_t)((pm * kLanes + lane) * 8);
        if constexpr (RG) x.p32off = (uint32_t)((((p & (kRingR - 1)) * kLanes) + lane) * 8);
    };
    // The steps of chunk ch over its present days, on one of the three paths (uniform in the wave).
    // (Round 5 measured two consecutive days with the same present lanes fused into one
    // straight-line step -- both days' ring reads in one batch: slower, 2.76 vs 2.54 ms at 1,250
    // assets, 4.2 vs 3.9 at 3,000; the scheduler kept day s's output chain ahead of day s + 1's
    // updates and the pair test cost more than it overlapped.  DESIGN.md §4.)
    auto fast_chunk = [&](int ch, unsigned cb, unsigned& n8, unsigned& f8) {
        GLB double* row = a.out + (int64_t)ch * kChunk * a.lda;    // the chunk's first date row
        int p = pos, pm = pmod;
        st.par = ch & 1;
#pragma unroll 1
        for (int s = 0; s < kChunk; ++s, row += a.lda) {
            const bool pres = (cb >> s) & 1u;
            st.template reset<P::kOut.lo, P::kOut.hi>();   // absent lanes store NaN
            if (pres) {
                set_day(st, p, pm);
                st.gather();                          // every ring read of the step, then compute
                __builtin_amdgcn_sched_barrier(0);
                fast_day(st, s, n8, f8);
                ++p;
                pm = pm + 1 == kRing ? 0 : pm + 1;
            }
            if constexpr (P::kOut.lo != 0 || P::kOut.hi != 0) {
                if (__builtin_amdgcn_ballot_w64(pres) != 0ull) {   // the whole wave: the day's stores
                    st.out = row;
                    st.template flush<P::kOut.lo, P::kOut.hi>();
                }
            }
        }
        pos = p;
        pmod = pm;
    };
    auto slow_chunk = [&](int ch, unsigned cb, bool warm, unsigned& n8, unsigned& f8) {
        GLB double* row = a.out + (int64_t)ch * kChunk * a.lda;
        int p = pos, pm = pmod;
        st.par = ch & 1;
        if (warm) {
            // warm-up windows: every observation of the lane so far in range (the first kClean of
            // a listing); the fast cores with the counts of a filling window.  Before p = 57 the
            // row holds NaN (ACCEL_56), so the masks need no per-column tracking there; from
            // p = 57 the lane is clean and the fast columns' own tracking applies.
#pragma unroll 1
            for (int s = 0; s < kChunk; ++s, row += a.lda) {
                const bool pres = (cb >> s) & 1u;
                st.template reset<P::kOut.lo, P::kOut.hi>();   // absent lanes store NaN
                if (pres) {
                    set_day(st, p, pm);
                    st.sday = s;
                    st.gather();
                    __builtin_amdgcn_sched_barrier(0);
                    const double c0 = st.template c<0>(), v0 = st.template v<0>();
                    // day 0: unused (no return yet)
                    if constexpr ((RT & 1ull) != 0) {
                        if constexpr (RG) st.r0 = st.rr[0];
                        else st.r0 = c0 / st.template c<1>() - 1;
                    }
                    if constexpr ((GC & 1ull) != 0) {
                        if constexpr (RG) st.g0 = st.gg[0];
                        else st.g0 = v0 / st.template v<1>() - 1;
                    }
                    st.anynan = st.anybad = p < kClean - 1;
                    if (S & kSerC) rn.C.fupd(c0);
                    if (S & kSerV) rn.V.fupd(v0);
                    if (S & kSerVP) rn.VP.fupd(v0);
                    if (S & kSerVC) rn.VC.fupd(v0 * c0);
                    if (p >= 1) {
                        if (S & kSerR) rn.R.fupd(st.r0);
                        if (S & kSerXY) {
                            rn.X.fupd(st.r0);
                            rn.Y.fupd(st.g0);
                            rn.XY.fupd(st.r0 * st.g0);
                        }
                    }
                    jobs.wstep(st);
                    n8 |= st.anynan ? 1u << s : 0u;
                    f8 |= st.anybad ? 1u << s : 0u;
                    ++p;
                    pm = pm + 1 == kRing ? 0 : pm + 1;
                }
                if constexpr (P::kOut.lo != 0 || P::kOut.hi != 0) {
                    if (__builtin_amdgcn_ballot_w64(pres) != 0ull) {   // the whole wave: the day's stores
                        st.out = row;
                        st.template flush<P::kOut.lo, P::kOut.hi>();
                    }
                }
            }
        } else {
#pragma unroll 1
            for (int s = 0; s < kChunk; ++s, row += a.lda) {
                const bool pres = (cb >> s) & 1u;
                st.template reset<P::kOut.lo, P::kOut.hi>();   // absent lanes store NaN
                if (pres) {
                    set_day(st, p, pm);
                    st.sday = s;
                    st.anynan = false;
                    st.anybad = false;
                    const double c0 = st.C(0), v0 = st.V(0);
                    if ((RT & 1ull) != 0) {
                        if constexpr (RG) {
                            st.r0 = st.Rr(0);                  // NaN on observation 0
                        } else {
                            const double r = c0 / st.C(1) - 1;
                            st.r0 = p >= 1 ? r : qnan();
                        }
                    }
                    if ((GC & 1ull) != 0) {
                        if constexpr (RG) {
                            st.g0 = st.Gr(0);
                        } else {
                            const double g = v0 / st.V(1) - 1;
                            st.g0 = p >= 1 ? g : qnan();
                        }
                    }
                    if (S & kSerC) rn.C.upd(c0);
                    if (S & kSerV) rn.V.upd(v0);
                    if (S & kSerVP) rn.VP.upd(pinf(v0));
                    if (S & kSerVC) rn.VC.upd(pinf(v0 * c0));
                    if (S & kSerR) rn.R.upd(pinf(st.r0));
                    if (S & kSerXY) {
                        const double X = pinf(st.r0 + 0 * st.g0), Y = pinf(st.g0 + 0 * st.r0);
                        rn.X.upd(X);
                        rn.Y.upd(Y);
                        rn.XY.upd(X * Y);
                    }
                    jobs.step(st);
                    n8 |= st.anynan ? 1u << s : 0u;
                    f8 |= st.anybad ? 1u << s : 0u;
                    ++p;
                    pm = pm + 1 == kRing ? 0 : pm + 1;
                }
                if constexpr (P::kOut.lo != 0 || P::kOut.hi != 0) {
                    if (__builtin_amdgcn_ballot_w64(pres) != 0ull) {   // the whole wave: the day's stores
                        st.out = row;
                        st.template flush<P::kOut.lo, P::kOut.hi>();
                    }
                }
            }
        }
        pos = p;
        pmod = pm;
    };
    // store this wave's partial words of the word that chunk ch ends (SGPR row base + lane offset,
    // as the output stores); slot: the mask-partial planes of this set or of a combiner
    auto store_words = [&](int ch, GLB uint64_t* np, GLB uint64_t* bp, u64 n, u64 f) {
        const int64_t wrow = (((int64_t)(ch * kChunk) >> 6) - w0) * a.lda;
        typedef unsigned v2u __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, n),
            __builtin_amdgcn_make_buffer_rsrc((void*)(np + wrow), 0, 0x7fffffff, 0x00020000),
            (int)voff, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, f),
            __builtin_amdgcn_make_buffer_rsrc((void*)(bp + wrow), 0, 0x7fffffff, 0x00020000),
            (int)voff, 0, 0);
    };
    // the split correlations this wave combines: chunk ch's num / den (written by the CorrM /
    // CorrV waves before the barrier that ended chunk ch) -> the corr column's rows of chunk ch
    // (NaN where the lane is absent), its NaN bits into the combiner's own partial words
    auto combine = [&](int ch, unsigned cb) {
        if constexpr (KC != 0) {
            const LDS SmemRG* rg = (const LDS SmemRG*)smp;
            const int par = ch & 1, sh = (ch * kChunk) & 63;
#pragma unroll
            for (int k = 0; k < kCombs; ++k) {
                if (!((KC >> k) & 1u)) continue;
                const int col = comb_col(k), xs = comb_slot(k);
                GLB double* row = a.out + (int64_t)ch * kChunk * a.lda;
                unsigned n8 = 0u, f8 = 0u;
                // the chunk's 8 quotients are independent: all reads and divisions first, so
                // their latencies overlap (round 5: a one-day-at-a-time loop made a combining
                // wave the longest of its workgroup); absent lanes' quotients are discarded
                double xq[kChunk];
#pragma unroll
                for (int s = 0; s < kChunk; ++s) {
                    const bool pres = (cb >> s) & 1u;
                    const double x = rg->xnum[xs][par][s][lane] / rg->xden[xs][par][s][lane];
                    xq[s] = pres ? x : qnan();
                    n8 |= (pres && x != x) ? 1u << s : 0u;
                    f8 |= (pres && !__builtin_isfinite(x)) ? 1u << s : 0u;
                }
#pragma unroll
                for (int s = 0; s < kChunk; ++s, row += a.lda) {
                    if (__builtin_amdgcn_ballot_w64((cb >> s) & 1u) != 0ull) {
                        st.out = row;
                        st.store1(col, xq[s]);
                    }
                }
                cnb[k] |= (u64)n8 << sh;
                cfb[k] |= (u64)f8 << sh;
                if (sh + kChunk == 64 || ch + 1 == nch) {
                    store_words(ch, a.cnanpart + k * a.pstride, a.cbadpart + k * a.pstride,
                                cnb[k], cfb[k]);
                    cnb[k] = 0ull;
                    cfb[k] = 0ull;
                }
            }
        }
    };
    // chunk ch done: its day bits into the word masks, stored at each word end (masks_kernel
    // ORs the job waves' partials); then the chunk barrier
    auto chunk_end = [&](int ch, unsigned n8, unsigned f8) {
        const int sh = (ch * kChunk) & 63;                 // chunk offset inside its word
        nb |= (u64)n8 << sh;
        fb |= (u64)f8 << sh;
        if (sh + kChunk == 64 || ch + 1 == nch) {          // word end: this wave's partial words
            store_words(ch, a.nanpart, a.badpart, nb, fb);
            nb = 0ull;
            fb = 0ull;
        }
#ifdef AFM_FP_PROFILE
        const long long tb = __builtin_readcyclecounter();
        lds_barrier();
        twait += __builtin_readcyclecounter() - tb;
#else
        lds_barrier();
#endif
    };
    int ch = c0;
    unsigned cb_prev = 0u;                                  // the previous chunk's presence bits
    auto is_clean = [&](int c) {
        return __builtin_amdgcn_ballot_w64(sm.okbyte[c & 1][lane] != 2) == 0ull;
    };
    while (ch < nch) {
        if (is_clean(ch)) {
            // a run of chunks that are clean for the whole wave.  Its first chunk is peeled off
            // the hot loop and followed by a vmcnt(0): a register whose load (a spill reload of
            // the slow paths, the state restore) is still in flight at a loop head makes the
            // compiler wait on vmcnt inside that loop -- and vmcnt counts this wave's output
            // stores too, so that wait would drain them on every step
            {
                unsigned n8 = 0u, f8 = 0u;
                const unsigned cb = (unsigned)sm.cbyte[ch & 1][lane];
                if (ch > c0) combine(ch - 1, cb_prev);
                fast_chunk(ch, cb, n8, f8);
                cb_prev = cb;
                chunk_end(ch, n8, f8);
                ++ch;
            }
            __builtin_amdgcn_s_waitcnt(kWaitVm0);
            while (ch < nch && is_clean(ch)) {              // the hot loop
                unsigned n8 = 0u, f8 = 0u;
                const unsigned cb = (unsigned)sm.cbyte[ch & 1][lane];
                combine(ch - 1, cb_prev);
                fast_chunk(ch, cb, n8, f8);
                cb_prev = cb;
                chunk_end(ch, n8, f8);
                ++ch;
            }
        } else {                                            // one warm or general chunk
            const int okl = sm.okbyte[ch & 1][lane];
            const bool warm = __builtin_amdgcn_ballot_w64(okl == 0) == 0ull;
            unsigned n8 = 0u, f8 = 0u;
            const unsigned cb = (unsigned)sm.cbyte[ch & 1][lane];
            if (ch > c0) combine(ch - 1, cb_prev);
            slow_chunk(ch, cb, warm, n8, f8);
            cb_prev = cb;
            chunk_end(ch, n8, f8);
            ++ch;
        }
    }
    combine(nch - 1, cb_prev);          // the last chunk (its num / den: before the last barrier)
    if (stp) {
        JobState<P> js;
        js.jobs = jobs;
        js.rn = rn;
        js.pos = pos;
        js.pmod = pmod;
        state_io(stp, js, lane, true);
    }
#ifdef AFM_FP_PROFILE
    if (lane == 0) {
        const long long tot = __builtin_readcyclecounter() - tstart;
        const int jw = a.jw;
        const int slot = a.pslot;
        const long long tend = (long long)__builtin_amdgcn_s_memrealtime();
        g_wave_cycles[(slot * jw + wave) * 4 % (1 << 16)] = tot;
        g_wave_cycles[((slot * jw + wave) * 4 + 1) % (1 << 16)] = twait;
        g_wave_cycles[((slot * jw + wave) * 4 + 2) % (1 << 16)] = treal;
        g_wave_cycles[((slot * jw + wave) * 4 + 3) % (1 << 16)] = tend;
    }
#endif
}

// words of one wave's slab-carry state (the largest job set's JobState, or a loader's rings)
template <class P> constexpr int state_words() { return (int)((sizeof(JobState<P>) + 7) / 8); }
constexpr int cmax(int a, int b) { return a > b ? a : b; }
template <class Part, int K = 0>
constexpr int part_state_words() {
    if constexpr (K == Part::kSets) return loader_state_words<Part::kRG>();
    else return cmax(state_words<typename Part::template Set<K>::type>(), part_state_words<Part, K + 1>());
}
constexpr int kStateWords = cmax(cmax(part_state_words<PartC>(), part_state_words<PartS>()),
                                 part_state_words<PartT>());

// Job set k of a partition on this wave (a uniform branch chain; every set's code is inlined)
template <class Part, int K = 0>
__device__ __forceinline__ void dispatch_set(int k, const Args& a, LDS Smem* sm, int wave, int lane,
                                             int64_t block, GLB double* stp) {
    if constexpr (K < Part::kSets) {
#ifdef AFM_FP_ONLY   // instruction census (tools/pack_census.sh): one job set's code only
        if (K == AFM_FP_ONLY && k == K) {
#else
        if (k == K) {
#endif
            run_wave<typename Part::template Set<K>::type, Part::kRG>(a, sm, 0, wave, lane, block, stp);
            return;
        }
        dispatch_set<Part, K + 1>(k, a, sm, wave, lane, block, stp);
    }
}

// TYPES workgroups per block, each with J = kSets / TYPES job waves (job sets [J*type, J*type+J))
// and a loader wave.  PAIR (PartC only): one workgroup runs TWO such items (two rings, 2 x (J + 1)
// waves), items ordered type-major so a pair shares its job sets.  At 10k assets the 3-way split
// has 471 items of 6 waves and 78 KB of LDS; at 168 VGPRs (3 waves / SIMD) two separate 6-wave
// workgroups rarely co-reside on a CU (their waves land 2-2-1-1 on the SIMDs), so half of them ran
// in a second round; paired, 236 workgroups of 12 waves (3 per SIMD, 156 KB LDS) are all resident.
// Paired 3-way launch: job set k (0-4) or the loader (5) at wave position k of each half.  Wave
// w of a workgroup issues on SIMD w % 4, so positions 0, 2, 4 of the two halves share SIMDs 0 and
// 2 three to a SIMD, and positions 1, 3 share SIMDs 1 and 3 with the loaders (PartC puts the light
// sets at 0, 2, 4).  PartS: one 140-KB workgroup per CU, J + 1 <= 11 waves.
// waves per SIMD a launch shape needs resident (the VGPR budget)
template <class Part, int TYPES, bool PAIR>
constexpr int waves_per_simd() {
    constexpr int w = (Part::kSets / TYPES + 1) * (PAIR ? 2 : 1);
    if constexpr (Part::kRG) return (w + 3) / 4;          // one workgroup per CU
    return w >= 12 ? (w + 3) / 4 : 2;
}
template <class Part>
constexpr int smem_bytes() { return Part::kRG ? (int)sizeof(SmemRG) : (int)sizeof(Smem); }

template <class Part, int TYPES, bool PAIR>
__global__ __launch_bounds__(kLanes * (Part::kSets / TYPES + 1) * (PAIR ? 2 : 1)) __attribute__((amdgpu_waves_per_eu(waves_per_simd<Part, TYPES, PAIR>())))
void factor_panel_kernel(Args a) {
    constexpr int J = Part::kSets / TYPES;
    static_assert(!(PAIR && Part::kRG), "paired items: PartC only");
    // dynamic LDS: with a static size the compiler pads the VGPR allocation of the split
    // variants up to what it thinks the LDS occupancy allows
    extern __shared__ double sm_dyn[];
    const int lane = threadIdx.x & (kLanes - 1);
    const int wall = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int half = PAIR ? (wall >= J + 1 ? 1 : 0) : 0;
    const int pos = wall - half * (J + 1);
    LDS Smem* sm = (LDS Smem*)sm_dyn + half;
    int type;
    int64_t block;
    if (PAIR) {
        const int64_t item = 2 * (int64_t)blockIdx.x + half;
        if (item >= (int64_t)a.nblk * TYPES) { idle_wave(a); return; }
        type = (int)(item / a.nblk);
        block = item % a.nblk;
    } else {
        type = (int)(blockIdx.x % TYPES);
        block = blockIdx.x / TYPES;
    }
    // job index of this wave (J = the loader)
    const int wave = pos;
    const int ltid = (int)threadIdx.x - half * (J + 1) * kLanes;
    if (ltid < 128) sm->rtab[ltid] = 1.0 / (double)ltid;
    // (the loader's first barrier also publishes rtab)
    // this wave's slab-carry state slot
    GLB double* stp = a.state ? a.state + (((block * TYPES + type) * (J + 1) + wave) *
                                           (int64_t)kStateWords * kLanes) : nullptr;
    if (wave == J) { load_wave<Part::kRG>(a, sm, lane, block, stp); return; }
    // this set's partial-mask planes (keeps the type out of the job waves' registers); the
    // combiners' planes follow the kSets sets'
    Args at = a;
    const int64_t w0 = ((int64_t)a.c0 * kChunk) >> 6;
    at.pstride = ((a.t1 + 63) / 64 - w0) * a.lda;
    const int64_t po = (int64_t)(type * J + wave) * at.pstride;
    at.nanpart = a.nanpart + po;
    at.badpart = a.badpart + po;
    at.cnanpart = a.nanpart + (int64_t)Part::kSets * at.pstride;
    at.cbadpart = a.badpart + (int64_t)Part::kSets * at.pstride;
#ifdef AFM_FP_PROFILE
    at.pslot = (int)(block * TYPES + type);          // profile slot of this item
    at.jw = J;
#endif
    dispatch_set<Part>(type * J + wave, at, sm, wave, lane, block, stp);
}

// nanfree = present & no type flagged a NaN; finite = present & no type flagged a non-finite
__global__ __launch_bounds__(256) void masks_kernel(int64_t nwords, int64_t lda, int types,
                                                    const uint64_t* vbits, const uint64_t* nanpart,
                                                    const uint64_t* badpart, uint64_t* nanfree,
                                                    uint64_t* finite) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t n = nwords * lda;
    if (i >= n) return;
    u64 nm = 0ull, bm = 0ull;
    for (int t = 0; t < types; ++t) {
        nm |= nanpart[t * n + i];
        bm |= badpart[t * n + i];
    }
    const u64 v = vbits[i];
    nanfree[i] = v & ~nm;
    if (finite) finite[i] = v & ~bm;
}

// target = excess_ret1d.shift(-1), tmr_ret1d = ret1d.shift(-1) (No-talib.py:90-91): the value of
// the asset's NEXT present day, NaN on its last one.  One thread per (asset, 64-day presence
// word): the word is walked backwards carrying the next present day's pair, so every load and
// store is a coalesced row segment (lanes = consecutive assets, one date) and the loads of a
// 16-day group are issued together.  The pair that enters a word from the right is the first
// present day of a later word.  Only present cells of [t_begin, t_end) are written.
__global__ __launch_bounds__(256) void labels_kernel(int64_t T, int64_t t_begin, int64_t t_end,
                                                     int64_t lda, const double* excess,
                                                     const double* ret1d, const uint64_t* vbits,
                                                     double* target, double* tmr) {
    const int64_t a = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (a >= lda) return;
    const int64_t c = (t_begin >> 6) + blockIdx.y;
    const int64_t nch = (T + 63) / 64;
    const u64 w = vbits[c * lda + a];
    if (!w) return;
    // the first present day after this word
    double ne = __builtin_nan(""), nr = __builtin_nan("");
    for (int64_t cc = c + 1; cc < nch; ++cc) {
        const u64 x = vbits[cc * lda + a];
        if (x) {
            const int64_t tn = cc * 64 + __builtin_ctzll(x);
            ne = excess[tn * lda + a];
            nr = ret1d[tn * lda + a];
            break;
        }
    }
    const int64_t d0 = c * 64;
    const int s_lo = t_begin > d0 ? (int)(t_begin - d0) : 0;
    const int s_hi = t_end - d0 < 64 ? (int)(t_end - d0) : 64;     // write [s_lo, s_hi)
    for (int g = 48; g >= 0; g -= 16) {
        if (!((w >> g) & 0xffffull)) continue;
        double e[16], r[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {                // rows past T are never present
            const int64_t t = d0 + g + j;
            const int64_t tc = t < T ? t : T - 1;
            e[j] = excess[tc * lda + a];
            r[j] = ret1d[tc * lda + a];
        }
#pragma unroll
        for (int j = 15; j >= 0; --j) {
            const int s = g + j;
            if ((w >> s) & 1ull) {
                if (s >= s_lo && s < s_hi) {
                    const int64_t cell = (d0 + s) * lda + a;
                    target[cell] = ne;
                    tmr[cell] = nr;
                }
                ne = e[j];
                nr = r[j];
            }
        }
    }
}

// out = in without each asset's last present day: the rows whose shift(-1) labels (target,
// tmr_ret1d, No-talib.py:90-91) are NaN.  One thread per asset; words copied coalesced.
// words [c0, c1) of out; the last observation from all nwords words of vbits
__global__ __launch_bounds__(256) void drop_last_obs_kernel(int64_t nwords, int64_t lda,
                                                            const uint64_t* vbits,
                                                            const uint64_t* in, uint64_t* out,
                                                            int64_t c0, int64_t c1) {
    const int64_t a = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (a >= lda) return;
    int64_t last = -1;
    for (int64_t c = nwords - 1; c >= 0 && last < 0; --c) {
        const u64 w = vbits[c * lda + a];
        if (w) last = c * 64 + 63 - __builtin_clzll(w);
    }
    for (int64_t c = c0; c < c1; ++c) {
        u64 w = in[c * lda + a];
        if (last >= 0 && (last >> 6) == c) w &= ~(1ull << (last & 63));
        out[c * lda + a] = w;
    }
}

}  // namespace
}  // namespace afm

#ifdef AFM_FP_PROFILE
extern "C" int afm_debug_wave_cycles(long long* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(afm::g_wave_cycles), sizeof(long long) * n) ==
                   hipSuccess ? 0 : -1;
}
#endif

// The launch shape: a partition and its workgroups per block (TYPES), as one code -- PartC:
// 1, 3, 5 or 15; PartS: 100 + TYPES with TYPES = 10, 6, 5 or 3 (J = 3, 5, 6, 10 job waves per
// workgroup); PartT: 206 (TYPES = 6, J = 10; J = 5 / 6 measured slower than PartS at every size,
// profiles/r5_rt_partitions.txt, and are not built).  (The option factor_split takes the same
// codes.)
//  * PartS / PartT while their 140-KB workgroups (one per CU) all fit the device at once: the
//    N = 8 shard (20 blocks) PartS J = 3 (one job wave per SIMD), the N = 4 shard (40 blocks)
//    PartT J = 10, configs B / D (47 blocks) PartS J = 6, the N = 2 shard (79 blocks) PartS J = 10.
//  * PartC otherwise (config C, 157 blocks): the most job-set splits whose 78-KB workgroups are
//    all resident, two per CU; 3 at least (the unsplit 16-wave workgroup caps the waves at 128
//    VGPRs, below what the job waves need for the fast step); extra 3-way workgroups queue.
static int factor_types(afm_ctx* ctx, int64_t nblk) {
    if (ctx->factor_split) return ctx->factor_split;               // option factor_split
    const int64_t ncu = afm_ctx_cus(ctx);
    // PartS with one job wave per SIMD while that fits (up to 25 blocks: the N = 8 shard); then
    // PartT with 10 job waves per workgroup (26-42 blocks: the N = 4 shard); then PartS again
    // (measured, profiles/r5_rt_partitions.txt: at 1,250 assets PartS 2.49 ms vs PartT 2.74-3.01,
    // at 2,500 PartT 3.27 vs PartS 3.63)
    if (nblk * 10 <= ncu) return 110;
    if (nblk * 6 <= ncu) return 206;
    for (int t : {5, 3})
        if (nblk * t <= ncu) return 100 + t;
    int types = 3;
    for (int t : {5, 15})
        if (nblk * t <= 2 * ncu) types = t;
    return types;
}

// a launch code is a split of its partition's job sets: J job waves + a loader per workgroup
template <class Part>
static constexpr bool split_ok(int types) {
    return types >= 1 && Part::kSets % types == 0 && Part::kSets / types + 1 <= 16 &&
           (!Part::kRG || Part::kSets / types + 1 <= 11);
}
template <class Part, int TYPES, bool PAIR>
static int launch_split(afm_ctx* ctx, int64_t nblk, const afm::Args& a) {
    if constexpr (!split_ok<Part>(TYPES)) {
        (void)ctx; (void)nblk; (void)a;
        afm_set_error("factor kernel: factor_split is not a split of the job sets");
        return AFM_E_ARG;
    } else {
        constexpr int J = Part::kSets / TYPES;
        const int bytes = afm::smem_bytes<Part>() * (PAIR ? 2 : 1);    // > 64 KB: opt in
        AFM_HIP(afm_lds_opt_in(ctx, (const void*)afm::factor_panel_kernel<Part, TYPES, PAIR>, bytes));
        const int64_t items = nblk * TYPES;
        const dim3 grid((unsigned)(PAIR ? (items + 1) / 2 : items));
        hipLaunchKernelGGL((afm::factor_panel_kernel<Part, TYPES, PAIR>), grid,
                           dim3(64 * (J + 1) * (PAIR ? 2 : 1)), bytes, ctx->stream, a);
        AFM_HIP(hipGetLastError());
        return AFM_OK;
    }
}
// mask partials of a launch code
static int code_parts(int code) {
    return code > 200 ? afm::nparts<afm::PartT>()
                      : code > 100 ? afm::nparts<afm::PartS>() : afm::nparts<afm::PartC>();
}
static int code_types(int code) { return code % 100; }
static int code_sets(int code) {
    return code > 200 ? afm::PartT::kSets : code > 100 ? afm::PartS::kSets : afm::PartC::kSets;
}

// The factor kernel over the time slab [t0, t1) of the [T]-date series (t0 a multiple of 64;
// [0, T) = the whole series).  out / nanfree / finite hold the slab's dates only.  state: the
// carry between consecutive slabs (null for a whole series).
static int factors_slab(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda, int64_t t0, int64_t t1,
                        const double* close, const double* volume, const double* ret1d,
                        const double* excess, const uint64_t* valid_bits, double* out,
                        uint64_t* nanfree_bits, uint64_t* finite_bits, double* state,
                        bool full = false, uint64_t* ext_part = nullptr) {
    // ext_part: the caller's buffer for the mask partials (afm_factors_part_words); the masks
    // are then left to afm_factor_masks_f64
    // full: out / nanfree / finite are the whole [T]-date panel and bit words (the slab's rows
    // and words written in place); else they hold the slab's dates only
    const int64_t nwords = (t1 - t0 + 63) / 64;                   // the slab's mask words
    if (state) {                     // the state layout depends on the split: keep it per series
        const int types_now = factor_types(ctx, (A + 63) / 64);
        std::lock_guard<std::mutex> lk(ctx->slab_mu);
        if (t0 == 0) {
            ctx->slab_types[state] = types_now;
        } else {
            const auto it = ctx->slab_types.find(state);
            if (it == ctx->slab_types.end()) {
                afm_set_error("factor slab: t0 > 0 continues a series whose state buffer was "
                              "never started at t0 = 0 on this context");
                return AFM_E_ARG;
            }
            if (it->second != types_now) {
                afm_set_error("factor slab: factor_split changed between slabs of one series "
                              "(the carried state was written under another split)");
                return AFM_E_ARG;
            }
        }
    }
    if (full) {                       // (null on the ext_part path: the masks come later)
        if (nanfree_bits) nanfree_bits += (t0 / 64) * lda;
        if (finite_bits) finite_bits += (t0 / 64) * lda;
    }
    const int64_t nblk = (A + 63) / 64;
    const int code = factor_types(ctx, nblk);
    const int types = code_types(code), nparts = code_parts(code);
    uint64_t* part = ext_part;        // per-job-wave mask partials (masks_kernel ORs them)
    if (!ext_part) {
        hipError_t e;
        part = (uint64_t*)afm_ctx_scratch(ctx, AFM_SCRATCH_FACTOR_PARTS,
                                          sizeof(uint64_t) * 2 * nparts * nwords * lda, &e);
        AFM_HIP(e);
    }
    afm::Args a;
    a.T = T;
    a.lda = lda;
    a.plane = (full ? T : t1 - t0) * lda;
    a.close = (const GLB double*)close;
    a.volume = (const GLB double*)volume;
    a.vbits = (const GLB uint64_t*)valid_bits;
    a.out = (GLB double*)(full ? out : out - t0 * lda);   // date t's row at a.out + t * lda
    a.nanpart = (GLB uint64_t*)part;
    a.badpart = (GLB uint64_t*)(part + nparts * nwords * lda);
    a.cnanpart = a.cbadpart = nullptr;
    a.pstride = 0;
    a.jw = 0;
    a.types = types;
    a.nblk = (int)nblk;
    a.pslot = 0;
    a.fast = 1;
    a.c0 = (int)(t0 / afm::kChunk);
    a.c1 = (int)((t1 + afm::kChunk - 1) / afm::kChunk);
    a.t1 = t1;
    a.state = (GLB double*)state;
    a.load_state = t0 > 0 ? 1 : 0;
    // paired 12-wave workgroups for the 3-way split (see factor_panel_kernel); options
    // factor_pair / factor_fast: the invariance tests' A/B
    const bool pair = ctx->factor_pair != 0;
    a.fast = ctx->factor_fast ? 1 : 0;
    int rc;
    using afm::PartC;
    using afm::PartS;
    using afm::PartT;
    switch (code) {                  // paired 2-item workgroups for the 3-way split (see the kernel)
        case 1: rc = launch_split<PartC, 1, false>(ctx, nblk, a); break;
        case 3: rc = pair ? launch_split<PartC, 3, true>(ctx, nblk, a)
                          : launch_split<PartC, 3, false>(ctx, nblk, a);
                break;
        case 5: rc = launch_split<PartC, 5, false>(ctx, nblk, a); break;
        case 15: rc = launch_split<PartC, 15, false>(ctx, nblk, a); break;
        case 103: rc = launch_split<PartS, 3, false>(ctx, nblk, a); break;
        case 105: rc = launch_split<PartS, 5, false>(ctx, nblk, a); break;
        case 106: rc = launch_split<PartS, 6, false>(ctx, nblk, a); break;
        case 110: rc = launch_split<PartS, 10, false>(ctx, nblk, a); break;
        case 206: rc = launch_split<PartT, 6, false>(ctx, nblk, a); break;
        default:
            afm_set_error("factor kernel: factor_split is not a split of the job sets");
            rc = AFM_E_ARG;
    }
    if (rc != AFM_OK) return rc;
    AFM_HIP(hipGetLastError());
    if (ext_part) return AFM_OK;      // (labels: this entry takes none, see the header)
    const int64_t nw = nwords * lda;
    // columns past A (lda padding) carry no presence: their mask words come from valid_bits
    // (zero there), and the factor kernel never ran on blocks past ceil(A/64)
    hipLaunchKernelGGL(afm::masks_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0,
                       ctx->stream, nwords, lda, nparts, valid_bits + (t0 / 64) * lda, part,
                       part + nparts * nw, nanfree_bits, finite_bits);
    AFM_HIP(hipGetLastError());
    if (excess) {                  // NULL: the caller runs afm_labels_f64 (e.g. on another stream)
        dim3 g2((unsigned)((lda + 255) / 256), (unsigned)((t1 - 1) / 64 - t0 / 64 + 1));
        hipLaunchKernelGGL(afm::labels_kernel, g2, dim3(256), 0, ctx->stream, T, t0, t1, lda,
                           excess, ret1d, valid_bits, (double*)a.out + 96 * a.plane,
                           (double*)a.out + 97 * a.plane);
        AFM_HIP(hipGetLastError());
    }
    return AFM_OK;
}

extern "C" int afm_factors_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda,
                               const double* close, const double* volume, const double* ret1d,
                               const double* excess, const uint64_t* valid_bits, double* out,
                               uint64_t* nanfree_bits, uint64_t* finite_bits) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(T > 0 && A > 0, "T and A must be positive");
    AFM_CHECK_ARG(lda >= A && lda % 64 == 0, "lda must be a multiple of 64 and >= A");
    AFM_CHECK_ARG(close && volume && valid_bits && out && nanfree_bits, "null buffer");
    AFM_CHECK_ARG((ret1d == nullptr) == (excess == nullptr),
                  "ret1d and excess are both given or both NULL");
    AFM_CHECK_ARG(T <= (int64_t)1 << 31, "T too large");
    return factors_slab(ctx, T, A, lda, 0, T, close, volume, ret1d, excess, valid_bits, out,
                        nanfree_bits, finite_bits, nullptr);
}

extern "C" int64_t afm_factors_state_bytes(afm_ctx* ctx, int64_t A) {
    if (!ctx || A <= 0) return -1;
    const int64_t nblk = (A + 63) / 64;
    const int code = factor_types(ctx, nblk);
    const int types = code_types(code);
    return nblk * types * (code_sets(code) / types + 1) * (int64_t)afm::kStateWords * 64 * 8;
}

extern "C" int afm_factors_slab_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda, int64_t t0,
                                    int64_t t1, const double* close, const double* volume,
                                    const double* ret1d, const double* excess,
                                    const uint64_t* valid_bits, double* out,
                                    uint64_t* nanfree_bits, uint64_t* finite_bits, double* state) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(T > 0 && A > 0, "T and A must be positive");
    AFM_CHECK_ARG(lda >= A && lda % 64 == 0, "lda must be a multiple of 64 and >= A");
    AFM_CHECK_ARG(close && volume && valid_bits && out && nanfree_bits, "null buffer");
    AFM_CHECK_ARG((ret1d == nullptr) == (excess == nullptr),
                  "ret1d and excess are both given or both NULL");
    AFM_CHECK_ARG(T <= (int64_t)1 << 31, "T too large");
    AFM_CHECK_ARG(0 <= t0 && t0 < t1 && t1 <= T && t0 % 64 == 0,
                  "need 0 <= t0 < t1 <= T with t0 a multiple of 64");
    AFM_CHECK_ARG(state != nullptr, "the slab state buffer is required");
    return factors_slab(ctx, T, A, lda, t0, t1, close, volume, ret1d, excess, valid_bits, out,
                        nanfree_bits, finite_bits, state);
}

extern "C" int afm_factors_range_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda, int64_t t0,
                                     int64_t t1, const double* close, const double* volume,
                                     const double* ret1d, const double* excess,
                                     const uint64_t* valid_bits, double* out,
                                     uint64_t* nanfree_bits, uint64_t* finite_bits, double* state) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(T > 0 && A > 0, "T and A must be positive");
    AFM_CHECK_ARG(lda >= A && lda % 64 == 0, "lda must be a multiple of 64 and >= A");
    AFM_CHECK_ARG(close && volume && valid_bits && out && nanfree_bits, "null buffer");
    AFM_CHECK_ARG((ret1d == nullptr) == (excess == nullptr),
                  "ret1d and excess are both given or both NULL");
    AFM_CHECK_ARG(T <= (int64_t)1 << 31, "T too large");
    AFM_CHECK_ARG(0 <= t0 && t0 < t1 && t1 <= T && t0 % 64 == 0 && (t1 % 64 == 0 || t1 == T),
                  "need 0 <= t0 < t1 <= T with t0 and t1 (unless T) multiples of 64");
    AFM_CHECK_ARG(state != nullptr, "the slab state buffer is required");
    return factors_slab(ctx, T, A, lda, t0, t1, close, volume, ret1d, excess, valid_bits, out,
                        nanfree_bits, finite_bits, state, true);
}

extern "C" int afm_labels_f64(afm_ctx* ctx, int64_t T, int64_t lda, int64_t t0, int64_t t1,
                              const double* excess, const double* ret1d,
                              const uint64_t* valid_bits, double* target, double* tmr) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(T > 0 && lda > 0 && lda % 64 == 0, "bad panel shape");
    AFM_CHECK_ARG(excess && ret1d && valid_bits && target && tmr, "null buffer");
    t0 = t0 < 0 ? 0 : t0;
    t1 = t1 > T ? T : t1;
    if (t1 <= t0) return AFM_OK;
    dim3 g2((unsigned)((lda + 255) / 256), (unsigned)((t1 - 1) / 64 - t0 / 64 + 1));
    hipLaunchKernelGGL(afm::labels_kernel, g2, dim3(256), 0, ctx->stream, T, t0, t1, lda, excess,
                       ret1d, valid_bits, target, tmr);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_drop_last_obs_bits(afm_ctx* ctx, int64_t T, int64_t lda,
                                      const uint64_t* valid_bits, const uint64_t* in_bits,
                                      uint64_t* out_bits) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(T > 0 && lda > 0 && lda % 64 == 0, "bad panel shape");
    AFM_CHECK_ARG(valid_bits && in_bits && out_bits, "null buffer");
    hipLaunchKernelGGL(afm::drop_last_obs_kernel, dim3((unsigned)((lda + 255) / 256)), dim3(256),
                       0, ctx->stream, (T + 63) / 64, lda, valid_bits, in_bits, out_bits,
                       (int64_t)0, (T + 63) / 64);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_drop_last_obs_bits_range(afm_ctx* ctx, int64_t T, int64_t lda,
                                            const uint64_t* valid_bits, const uint64_t* in_bits,
                                            uint64_t* out_bits, int64_t t0, int64_t t1) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(T > 0 && lda > 0 && lda % 64 == 0, "bad panel shape");
    AFM_CHECK_ARG(valid_bits && in_bits && out_bits, "null buffer");
    AFM_CHECK_ARG(0 <= t0 && t0 < t1 && t1 <= T && t0 % 64 == 0 && (t1 % 64 == 0 || t1 == T),
                  "need 0 <= t0 < t1 <= T with t0 and t1 (unless T) multiples of 64");
    hipLaunchKernelGGL(afm::drop_last_obs_kernel, dim3((unsigned)((lda + 255) / 256)), dim3(256),
                       0, ctx->stream, (T + 63) / 64, lda, valid_bits, in_bits, out_bits,
                       t0 / 64, (t1 + 63) / 64);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int64_t afm_factors_part_words(afm_ctx* ctx, int64_t A, int64_t lda, int64_t t0,
                                          int64_t t1) {
    if (!ctx || A <= 0 || lda < A || t1 <= t0) return -1;
    const int code = factor_types(ctx, (A + 63) / 64);
    return 2 * (int64_t)code_parts(code) * ((t1 - t0 + 63) / 64) * lda;
}

extern "C" int afm_factors_range_part_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda,
                                          int64_t t0, int64_t t1, const double* close,
                                          const double* volume, const uint64_t* valid_bits,
                                          double* out, double* state, uint64_t* part) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(T > 0 && A > 0, "T and A must be positive");
    AFM_CHECK_ARG(lda >= A && lda % 64 == 0, "lda must be a multiple of 64 and >= A");
    AFM_CHECK_ARG(close && volume && valid_bits && out && state && part, "null buffer");
    AFM_CHECK_ARG(T <= (int64_t)1 << 31, "T too large");
    AFM_CHECK_ARG(0 <= t0 && t0 < t1 && t1 <= T && t0 % 64 == 0 && (t1 % 64 == 0 || t1 == T),
                  "need 0 <= t0 < t1 <= T with t0 and t1 (unless T) multiples of 64");
    // (no bit-word pointers on this path: the masks come later, afm_factor_masks_f64)
    return factors_slab(ctx, T, A, lda, t0, t1, close, volume, nullptr, nullptr, valid_bits, out,
                        nullptr, nullptr, state, true, part);
}

extern "C" int afm_factor_masks_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda, int64_t t0,
                                    int64_t t1, const uint64_t* valid_bits, const uint64_t* part,
                                    uint64_t* nanfree_bits, uint64_t* finite_bits) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(T > 0 && A > 0 && lda >= A && lda % 64 == 0, "bad shape");
    AFM_CHECK_ARG(valid_bits && part && nanfree_bits, "null buffer");
    AFM_CHECK_ARG(0 <= t0 && t0 < t1 && t1 <= T && t0 % 64 == 0, "bad date range");
    const int code = factor_types(ctx, (A + 63) / 64);
    const int64_t nwords = (t1 - t0 + 63) / 64, nw = nwords * lda;
    const int nparts = code_parts(code);
    hipLaunchKernelGGL(afm::masks_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0,
                       ctx->stream, nwords, lda, nparts, valid_bits + (t0 / 64) * lda, part,
                       part + nparts * nw, nanfree_bits + (t0 / 64) * lda,
                       finite_bits ? finite_bits + (t0 / 64) * lda : nullptr);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

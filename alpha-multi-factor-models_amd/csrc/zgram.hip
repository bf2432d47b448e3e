// The regression stages of the reference chain on z-scored features, without materialising the
// z-scored planes (KKT Yuliang Jiang.py:446-458 feeding :582-612):
//
//   zstats_finalize  per (feature, asset): zs = {mu, 1/sigma} of the train-window groupby
//                    mean/std (zscore.hip computes mu/sigma pandas-exactly), asset_ok = every
//                    feature has a finite mean and sigma > 0 -- exactly the assets whose rows
//                    survive .replace([inf, -inf], nan).dropna() (KKT:452-454): any other asset
//                    has a NaN or +-inf z in every row of some column.
//   row_bits         word-wise AND of row masks, an asset mask and a date range (the split and
//                    dropna row sets of KKT:426-458 on the calendar grid).
//   zgram            per (date, asset block): partial Gram of Z = [1, z_1 .. z_p, y] with
//                    z = (x - mu) * (1/sigma) computed while staging, every entry on
//                    v_mfma_f64_16x16x4_f64 (the ones column and y ride in the 112-wide tile, so
//                    there is no VALU border sum).  Raw (unshifted) moments: the features are
//                    z-scores, centred by construction.
//   gram_merge       sums the block partials of a date over a FIXED pairwise tree
//                    ((b0 + b1) + (b2 + b3)) + ((b4 + b5) + (b6 + b7)).  A rank of a multi-GPU
//                    run owns a contiguous power-of-two run of blocks, merges its subtree, and the
//                    date's owner merges the subtree results: the same tree, so every GPU count
//                    produces bit-identical Grams (and everything downstream).
//   zpredict         pred = b0 + sum_j b_j z_j on the fly, skipping zero coefficients (exact:
//                    +-0 * finite z adds nothing), so a sparse Lasso reads only its support.
//
// Algorithmic work of zgram: rows * (p+2)(p+3) flops per date; bytes: 8(p+1) per
// row from HBM (+16 p per row of {mu, 1/sigma}, L2-resident per asset block: blocks map to XCDs).
#include "afm_internal.h"

#include <cstdlib>

#pragma clang fp contract(off)

namespace afm {
namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;
// LDS-qualified double: keeps ring accesses on ds_read / ds_write (a generic pointer to dynamic
// LDS would compile to flat loads, which wait on vmcnt and lgkmcnt together)
typedef __attribute__((address_space(3))) double lds_double;

constexpr int kZRS = 66;                     // LDS row stride (doubles): conflict-free fragments
constexpr int kZMaxSlots = 3;                // ring depth (2 when p + 4 staged rows do not fit 3x)
constexpr int kZLds = 160 * 1024 - 256;      // dynamic LDS budget of the ring
constexpr int kZProd = 8;                    // producer waves
constexpr int kZThreads = 13 * 64;           // 8 producers + up to 4 consumers + border wave
#ifndef AFM_ZG2_NCW                          // (A/B builds: tools/build_flags_variant.sh)
#define AFM_ZG2_NCW 3
#endif

// Shapes: NT 16-wide tiles (NT = 7: p + 2 <= 108, the 97-feature design; NT = 2: p + 2 <= 32,
// the FM30 design).  Consumer wave c owns tile pairs [c * PPW, (c + 1) * PPW) of the J-major
// upper-triangle list.
template <int NT>
struct ZCfg {
    static constexpr int NP = NT * (NT + 1) / 2;
    static constexpr int PE = NP * 256;                        // doubles of one partial
    static constexpr int NCW = NT == 7 ? 4 : AFM_ZG2_NCW;      // consumer waves
    // NT = 7: the columns of the last tile (96 .. p+1, at most 12) go to the border wave's VALU
    // sums; the MFMA consumers take the 21 pairs of tiles 0..5 -- 3 on wave 0 (which shares SIMD 0
    // with the border wave), 6 on each of waves 1..3.  NT = 2: all 3 pairs, one per wave.
    static constexpr bool BORDER = NT == 7;
    static constexpr int NMP = BORDER ? (NT - 1) * NT / 2 : NP;   // MFMA pairs
    static constexpr int NWAIT = NCW + (BORDER ? 1 : 0);          // waves that free a slot
    static constexpr int KMAX = NT == 7 ? 108 : 16 * NT;       // staged columns p + 2 <= KMAX
    static constexpr int MC = (KMAX + kZProd - 1) / kZProd;    // columns per producer wave
    static constexpr int q0(int cw) {
        return BORDER ? (cw == 0 ? 0 : 3 + 6 * (cw - 1)) : cw * ((NMP + NCW - 1) / NCW);
    }
    static constexpr int nq(int cw) {
        return BORDER ? (cw == 0 ? 3 : 6)
                      : (q0(cw) + (NMP + NCW - 1) / NCW <= NMP ? (NMP + NCW - 1) / NCW : NMP - q0(cw));
    }
};

template <int NT>
struct ZPairs {
    int I[ZCfg<NT>::NP], J[ZCfg<NT>::NP];
    constexpr ZPairs() : I(), J() {
        int q = 0;
        for (int j = 0; j < NT; ++j)
            for (int i = 0; i <= j; ++i) { I[q] = i; J[q] = j; ++q; }
    }
};

struct ZGramArgs {
    const double* base;      // factor planes: column c at base + c * col_stride, [T][lda]
    int64_t col_stride;
    int64_t lda;
    const int32_t* cols;     // [p] regressor planes
    const int32_t* zcols;    // [p] zs row of each regressor (null: row k for regressor k)
    int p;
    int ycol;                // regressand plane
    int zid;                 // zs identity row {0, 1} (the regressand)
    const double* zs;        // [rows][lda][2] {mu, 1/sigma}
    const uint64_t* bits;    // [ceil(T/64)][lda] rows used
    int64_t t0, nt;          // dates [t0, t0 + nt)
    int mode;                // 0: items (date, asset block); 1: items (row-block, date chunk)
    int nblk;                // mode 0: asset blocks
    int64_t blk0;            // first asset (multiple of 64)
    int64_t blk_assets;      // mode 0: assets per block (multiple of 64)
    int64_t a_end;           // assets >= a_end are absent
    int nrb;                 // mode 1: row-blocks from blk0
    int nchunk;              // mode 1: date chunks of [t0, t0 + nt)
    double* part;            // mode 0: [nt][nblk][PE]; mode 1: [nrb][nchunk][PE]
    int even;                // pad every item to an even slot count (zgram_produce_pairs)
};

// The ring: nslots slots of (p + 4) LDS rows (rows 0..p+1 staged, row p+2 stays zero: the
// fragment source of the padding features, row p+3: dump row of the dummy columns), dynamic
// LDS; counters in static LDS.
struct ZSmem {
    lds_double* tile;        // [nslots][p + 4][kZRS]
    int slot_elems;          // (p + 4) * kZRS
    int nslots;
    int ready[kZMaxSlots];
    int freed[kZMaxSlots];
};

__device__ __forceinline__ int lds_load_acq(int* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void wait_count(int* p, int target) {
    while (__builtin_amdgcn_readfirstlane(lds_load_acq(p)) < target) __builtin_amdgcn_s_sleep(1);
}
__device__ __forceinline__ void signal_count(int* p, int lane) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(p, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The row-block sequence of one workgroup: items blockIdx.x, + gridDim.x, ... (persistent).
//  mode 0: item = (date d, block b): the block's row-blocks (at least one) at date t0 + d;
//  mode 1: item = (row-block r, chunk c): row-block r at every date of chunk c (at least one
//          slot: an empty chunk stages one all-masked block).
// With g.even every item has an EVEN number of slots (an odd count gets one all-masked slot
// more): zgram_produce_pairs stages two buffers per loop iteration, never straddling two items.
// Every wave walks the same sequence; the item's last row-block flushes the consumers.
struct Seq {
    int item, nitems, stride;
    int t, a_lo;             // current row-block: date, first asset
    int masked;              // an all-masked slot (empty chunk, or the padding slot)
    int k, kend, kreal;      // position inside the item (row-block or date); real slots < kreal
    __device__ void start(const ZGramArgs& g) {
        if (g.mode == 0) {
            const int d = item / g.nblk, b = item - d * g.nblk;
            t = (int)g.t0 + d;
            const int lo = (int)g.blk0 + b * (int)g.blk_assets;
            int hi = lo + (int)g.blk_assets;
            if (hi > (int)g.a_end) hi = (int)g.a_end;
            const int n = hi > lo ? (hi - lo + 63) / 64 : 0;
            a_lo = lo;
            k = 0;
            kreal = n;
            kend = (n > 0 ? n : 1) + (g.even ? ((n > 0 ? n : 1) & 1) : 0);
        } else {
            const int r = item / g.nchunk, c = item - r * g.nchunk;
            const int c0 = (int)g.t0 + (int)(((int64_t)c * g.nt) / g.nchunk);
            const int c1 = (int)g.t0 + (int)(((int64_t)(c + 1) * g.nt) / g.nchunk);
            const int n = c1 > c0 ? c1 - c0 : 1;
            a_lo = (int)g.blk0 + r * 64;
            k = c0;
            kreal = c1;
            kend = c0 + n + (g.even ? (n & 1) : 0);
            t = c0;
        }
        masked = k >= kreal ? 1 : 0;
    }
    __device__ void init(const ZGramArgs& g) {
        stride = gridDim.x;
        nitems = g.mode == 0 ? (int)g.nt * g.nblk : g.nrb * g.nchunk;
        item = blockIdx.x;
        if (item < nitems) start(g);
    }
    __device__ bool valid() const { return item < nitems; }
    __device__ bool last() const { return k + 1 == kend; }
    __device__ int row_asset(int lane) const { return a_lo + lane; }
    __device__ void advance(const ZGramArgs& g) {
        if (k + 1 < kend) {
            ++k;
            masked = k >= kreal ? 1 : 0;
            if (g.mode == 0) a_lo += 64;
            else t = masked ? t : k;              // a padding slot keeps a real date (masked)
            return;
        }
        item += stride;
        if (item < nitems) start(g);
    }
};

// Producer wave pw stages tile rows k = pw + 8 j (k = 0: ones, 1..p: z features, p+1: y;
// larger k: a dummy load of y into the dump row p+3, so the loop has no per-column branch).
// x (HBM) is loaded two row-blocks ahead.  {mu, 1/sigma} (16 B per cell): mode 0 one row-block
// ahead, issued before the newer x loads (loads retire in order); mode 1 once per item -- the
// item keeps its 64 assets, so the row-block's statistics stay in registers across its dates.
// z = (x - mu) * rsig; masked-out rows stage exact zeros.
template <int NT, int MODE, bool ZS>
__device__ void zgram_produce(const ZGramArgs& g, ZSmem& sm, const int lane, const int pw) {
    constexpr int MC = ZCfg<NT>::MC;
    const int p = g.p;
    const int K = p + 2;
    const int lda = (int)g.lda;
    // plane and zs row of every column (SGPRs); the 64-bit addresses are re-derived at each load
    // (SALU work -- the asm keeps the compiler from hoisting 2 x MC 64-bit pointers into SGPRs)
    // (plane | zs row << 16: one SGPR per column)
    int pk[MC];
#pragma unroll
    for (int j = 0; j < MC; ++j) {
        const int k = pw + kZProd * j;
        const bool feat = k >= 1 && k <= p;
        const int pl = feat ? g.cols[k - 1] : g.ycol;
        const int zr = feat ? (g.zcols ? g.zcols[k - 1] : k - 1) : g.zid;
        pk[j] = __builtin_amdgcn_readfirstlane(pl | (zr << 16));
    }
    auto xsrc = [&](int j) {
        int q = pk[j];
        asm volatile("" : "+s"(q));
        return reinterpret_cast<const char*>(g.base + (int64_t)(q & 0xffff) * g.col_stride);
    };
    auto zsrc = [&](int j) {
        int q = pk[j];
        asm volatile("" : "+s"(q));
        return (unsigned)((q >> 16) * lda) * 16u;
    };
    const char* zb = reinterpret_cast<const char*>(g.zs);
    struct Buf {
        double x[MC];
        bool ok;
        unsigned zoff;
        int item;
    };
    Buf A, C;
    double mu[MC], rs[MC];
    int zitem = -1;
    Seq cur;
    cur.init(g);
    auto xload = [&](Buf& B) {
        const int t = cur.t;
        const int a = cur.row_asset(lane);
        const bool in = a < (int)g.a_end && !cur.masked;
        const int ac = in ? a : 0;
        B.ok = in && ((g.bits[(int64_t)(t >> 6) * lda + ac] >> (t & 63)) & 1ull);
        B.zoff = (unsigned)ac * 16u;
        B.item = cur.item;
        const unsigned off = (unsigned)(t * lda + ac) * 8u;
#pragma unroll
        for (int j = 0; j < MC; ++j) B.x[j] = *reinterpret_cast<const double*>(xsrc(j) + off);
    };
    auto zload = [&](const unsigned zoff) {
        if (!ZS) return;                             // raw columns: no statistics
#pragma unroll
        for (int j = 0; j < MC; ++j) {
            const double2 m = *reinterpret_cast<const double2*>(zb + zsrc(j) + zoff);
            mu[j] = m.x;
            rs[j] = m.y;
        }
    };
    int slot = 0, gen = 0;
    auto stage = [&](const Buf& B) {
        if (ZS && MODE == 1 && B.item != zitem) {    // a new item: its row-block's statistics
            zload(B.zoff);
            zitem = B.item;
        }
        wait_count(&sm.freed[slot], ZCfg<NT>::NWAIT * gen);
        lds_double* tb = sm.tile + slot * sm.slot_elems + lane;
#pragma unroll
        for (int j = 0; j < MC; ++j) {
            const int k = pw + kZProd * j;
            const int lrow = k < K ? k : p + 3;      // the dump row takes the dummy columns
            double v = ZS ? (B.x[j] - mu[j]) * rs[j] : B.x[j];   // y: identity row {0, 1}
            if (k == 0) v = 1.0;                     // the ones column (wave 0, j = 0)
            tb[lrow * kZRS] = B.ok ? v : 0.0;
        }
        signal_count(&sm.ready[slot], lane);
        if (++slot == sm.nslots) { slot = 0; ++gen; }
    };
    bool ha = cur.valid(), hc = false;
    if (ha) { xload(A); cur.advance(g); }
    if (MODE == 0 && ha) zload(A.zoff);
    hc = cur.valid();
    if (hc) { xload(C); cur.advance(g); }
    while (ha) {
        stage(A);
        if (MODE == 0 && hc) zload(C.zoff);          // next statistics first, then x two ahead
        ha = cur.valid();
        if (ha) { xload(A); cur.advance(g); }
        if (!hc) break;
        stage(C);
        if (MODE == 0 && ha) zload(A.zoff);
        hc = cur.valid();
        if (hc) { xload(C); cur.advance(g); }
    }
}

// zgram_produce with a prefetch the compiler's waits keep in flight (the per-date FM Grams:
// their producers are load-latency-bound, 3.9 -> 3.0 ms): every xload / zload issues its loads on
// every path and the presence word is tested only when staging -- a load consumed where it is
// issued makes the compiler wait for every outstanding load, the whole prefetch, right there.
// Items have an even slot count (g.even), so each iteration stages the pair (A, C) of one item.
// (The pooled Gram keeps zgram_produce: it is bound by the MFMA / staging serialisation on the
// SIMDs, and there the deeper prefetch measured slower, 11.1 -> 12.1 ms.)
template <int NT, int MODE, bool ZS>
__device__ void zgram_produce_pairs(const ZGramArgs& g, ZSmem& sm, const int lane, const int pw) {
    constexpr int MC = ZCfg<NT>::MC;
    const int p = g.p;
    const int K = p + 2;
    const int lda = (int)g.lda;
    // plane and zs row of every column (SGPRs); the 64-bit addresses are re-derived at each load
    // (SALU work -- the asm keeps the compiler from hoisting 2 x MC 64-bit pointers into SGPRs)
    // (plane | zs row << 16: one SGPR per column)
    int pk[MC];
#pragma unroll
    for (int j = 0; j < MC; ++j) {
        const int k = pw + kZProd * j;
        const bool feat = k >= 1 && k <= p;
        const int pl = feat ? g.cols[k - 1] : g.ycol;
        const int zr = feat ? (g.zcols ? g.zcols[k - 1] : k - 1) : g.zid;
        pk[j] = __builtin_amdgcn_readfirstlane(pl | (zr << 16));
    }
    auto xsrc = [&](int j) {
        int q = pk[j];
        asm volatile("" : "+s"(q));
        return reinterpret_cast<const char*>(g.base + (int64_t)(q & 0xffff) * g.col_stride);
    };
    auto zsrc = [&](int j) {
        int q = pk[j];
        asm volatile("" : "+s"(q));
        return (unsigned)((q >> 16) * lda) * 16u;
    };
    const char* zb = reinterpret_cast<const char*>(g.zs);
    struct Buf {
        double x[MC];
        uint32_t word;           // the half presence word holding the row's bit, tested when
        bool in, valid;          // staging: a load consumed at issue would make the compiler
        unsigned zoff;           // wait for every outstanding load (the whole prefetch) there
        int t, item;
    };
    Buf A, C;
    double mu[MC], rs[MC];
    Seq cur;
    cur.init(g);
    // Every xload / zload issues its loads on every path (a finished sequence or a masked slot
    // reads the first cell): with the same loads in every iteration the compiler's waits before
    // a stage cover only that buffer, and the younger prefetch stays in flight.
    auto xload = [&](Buf& B) {
        const bool v = cur.valid();
        const int a = cur.row_asset(lane);
        const bool in = v && !cur.masked && a < (int)g.a_end;
        const int ac = in ? a : 0, tl = in ? cur.t : 0;
        B.valid = v;
        B.in = in;
        B.t = cur.t;
        B.item = v ? cur.item : -1;
        B.zoff = (unsigned)ac * 16u;
        B.word = reinterpret_cast<const uint32_t*>(g.bits)[((int64_t)(tl >> 6) * lda + ac) * 2 +
                                                           ((tl >> 5) & 1)];
        const unsigned off = (unsigned)(tl * lda + ac) * 8u;
#pragma unroll
        for (int j = 0; j < MC; ++j) B.x[j] = *reinterpret_cast<const double*>(xsrc(j) + off);
        if (v) cur.advance(g);
    };
    auto zload = [&](const unsigned zoff) {
        if (!ZS) return;                             // raw columns: no statistics
#pragma unroll
        for (int j = 0; j < MC; ++j) {
            const double2 m = *reinterpret_cast<const double2*>(zb + zsrc(j) + zoff);
            mu[j] = m.x;
            rs[j] = m.y;
        }
    };
    int slot = 0, gen = 0;
    auto stage = [&](const Buf& B) {
        wait_count(&sm.freed[slot], ZCfg<NT>::NWAIT * gen);
        lds_double* tb = sm.tile + slot * sm.slot_elems + lane;
        const bool ok = B.in && ((B.word >> (B.t & 31)) & 1u);
#pragma unroll
        for (int j = 0; j < MC; ++j) {
            const int k = pw + kZProd * j;
            const int lrow = k < K ? k : p + 3;      // the dump row takes the dummy columns
            double v = ZS ? (B.x[j] - mu[j]) * rs[j] : B.x[j];   // y: identity row {0, 1}
            if (k == 0) v = 1.0;                     // the ones column (wave 0, j = 0)
            tb[lrow * kZRS] = ok ? v : 0.0;
        }
        signal_count(&sm.ready[slot], lane);
        if (++slot == sm.nslots) { slot = 0; ++gen; }
    };
    xload(A);
    if (MODE == 0) zload(A.zoff);
    xload(C);
    while (A.valid) {                                // one item per iteration (even slot count)
        // mode 1: the item keeps its 64 assets -- its statistics stay in registers for its dates
        if (MODE == 1) zload(A.zoff);
        const int item = A.item;
        do {
            stage(A);
            if (MODE == 0) zload(C.zoff);            // next statistics first, then x two ahead
            xload(A);
            stage(C);
            if (MODE == 0) zload(A.zoff);
            xload(C);
        } while (A.valid && A.item == item);
    }
}

// Consumer wave CW: its tile pairs; fragments of the tiles they touch, two sets in ping-pong; an
// item's last row-block flushes the accumulators to the item's partial.
template <int NT, int CW>
__device__ void zgram_consume(const ZGramArgs& g, ZSmem& sm, const int lane) {
    using Cf = ZCfg<NT>;
    constexpr ZPairs<NT> tab{};
    constexpr int Q0 = Cf::q0(CW);
    constexpr int NQ = Cf::nq(CW);
    constexpr int THI = tab.J[Q0 + NQ - 1] + 1;                // tiles [0, THI) are touched
    const int fi = lane & 15, kk = lane >> 4;
    const int p = g.p;
    int lrow[NT];                            // LDS row of tile t for this lane (padding: zero row)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int f = t * 16 + fi;
        lrow[t] = f <= p + 1 ? f : p + 2;
    }
    d4 acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
    int slot = 0, gen = 1;
    Seq cur;
    for (cur.init(g); cur.valid(); cur.advance(g)) {
        wait_count(&sm.ready[slot], kZProd * gen);
        const lds_double* tb = sm.tile + slot * sm.slot_elems;
        double fa[NT], fb[NT];
        auto ld = [&](double (&f)[NT], int it) {
            const int a = it * 4 + kk;
#pragma unroll
            for (int t = 0; t < THI; ++t) f[t] = tb[lrow[t] * kZRS + a];
        };
        auto step = [&](const double (&f)[NT]) {
#pragma unroll
            for (int q = 0; q < NQ; ++q)
                acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(f[tab.I[Q0 + q]], f[tab.J[Q0 + q]],
                                                              acc[q], 0, 0, 0);
        };
        // k-step it+1's fragments are requested before k-step it's MFMAs
        ld(fa, 0);
#pragma unroll
        for (int it = 0; it < 16; it += 2) {
            ld(fb, it + 1);
            step(fa);
            if (it + 2 < 16) ld(fa, it + 2);
            step(fb);
        }
        signal_count(&sm.freed[slot], lane);
        if (++slot == sm.nslots) { slot = 0; ++gen; }
        if (cur.last()) {
            double* out = g.part + (int64_t)cur.item * Cf::PE + Q0 * 256 + lane;
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
#pragma unroll
                for (int r = 0; r < 4; ++r) out[(q * 4 + r) * 64] = acc[q][r];
                acc[q] = d4{0.0, 0.0, 0.0, 0.0};
            }
        }
    }
}

// The border wave (NT = 7): the Gram columns b = 96 .. p+1 (at most 12; p = 97: z_96, z_97, y)
// against every column c, as VALU sums over the staged rows -- lanes own columns c = lane,
// lane + 64, the border values are broadcast reads.  It shares SIMD 0 with the lightest MFMA
// consumer: f64 VALU and MFMA issue from separate pipes.  An item's last row-block flushes the
// sums into the partial's (c / 16, 6) tile pairs in the MFMA C/D layout, so the trees and the
// final symmetric write are unchanged.
__device__ __forceinline__ double rdlane_d(double v, int l) {     // l uniform
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

template <int NT, int NB>
__device__ void zgram_border(const ZGramArgs& g, ZSmem& sm, const int lane) {
    constexpr ZPairs<NT> tab{};
    const int K = g.p + 2;
    double acc[2][NB];
#pragma unroll
    for (int cc = 0; cc < 2; ++cc)
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[cc][b] = 0.0;
    int slot = 0, gen = 1;
    Seq cur;
    for (cur.init(g); cur.valid(); cur.advance(g)) {
        wait_count(&sm.ready[slot], kZProd * gen);
        // per row: the lane's two column values, and the NB border values as uniform-address
        // (broadcast) reads -- all independent of the sums, so an unrolled group is in flight
        const lds_double* tb = sm.tile + slot * sm.slot_elems;
        const lds_double* c0 = tb + lane * kZRS;
        const lds_double* c1 = tb + (lane + 64 < K ? lane + 64 : g.p + 2) * kZRS;  // zero row
        const lds_double* bb = tb + 96 * kZRS;
#pragma unroll 8
        for (int r = 0; r < 64; ++r) {
            const double x0 = c0[r], x1 = c1[r];
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                const double zb = bb[b * kZRS + r];
                acc[0][b] = __builtin_fma(x0, zb, acc[0][b]);
                acc[1][b] = __builtin_fma(x1, zb, acc[1][b]);
            }
        }
        signal_count(&sm.freed[slot], lane);
        if (++slot == sm.nslots) { slot = 0; ++gen; }
        if (cur.last()) {
            double* out = g.part + (int64_t)cur.item * ZCfg<NT>::PE;
#pragma unroll
            for (int cc = 0; cc < 2; ++cc) {
                const int c = lane + 64 * cc;
                if (c < K) {
                    const int ti = c >> 4, w = c & 15;
                    int q = 0;                                     // pair (ti, 6)
#pragma unroll
                    for (int qq = 0; qq < ZCfg<NT>::NP; ++qq)
                        if (tab.I[qq] == ti && tab.J[qq] == NT - 1) q = qq;
                    const int r4 = w >> 2, lrow = (w & 3) * 16;
#pragma unroll
                    for (int b = 0; b < NB; ++b) out[q * 256 + r4 * 64 + lrow + b] = acc[cc][b];
                }
#pragma unroll
                for (int b = 0; b < NB; ++b) acc[cc][b] = 0.0;
            }
        }
    }
}

// the border wave for any border width 1..12 (the pooled design has 3: z_96, z_97, y)
template <int NT>
__device__ void zgram_border_any(const ZGramArgs& g, ZSmem& sm, const int lane) {
    switch (g.p + 2 - 96) {
        case 1: zgram_border<NT, 1>(g, sm, lane); break;
        case 2: zgram_border<NT, 2>(g, sm, lane); break;
        case 3: zgram_border<NT, 3>(g, sm, lane); break;
        case 4: zgram_border<NT, 4>(g, sm, lane); break;
        case 5: zgram_border<NT, 5>(g, sm, lane); break;
        case 6: zgram_border<NT, 6>(g, sm, lane); break;
        case 7: zgram_border<NT, 7>(g, sm, lane); break;
        case 8: zgram_border<NT, 8>(g, sm, lane); break;
        case 9: zgram_border<NT, 9>(g, sm, lane); break;
        case 10: zgram_border<NT, 10>(g, sm, lane); break;
        case 11: zgram_border<NT, 11>(g, sm, lane); break;
        case 12: zgram_border<NT, 12>(g, sm, lane); break;
        default: zgram_border<NT, 0>(g, sm, lane); break;   // no border columns: just free slots
    }
}

template <int NT, int MODE, bool ZS>
__global__ __launch_bounds__(kZThreads, 1) void zgram_kernel(ZGramArgs g, int nslots) {
    extern __shared__ __attribute__((aligned(16))) double ring[];
    __shared__ ZSmem sm;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int se = (g.p + 4) * kZRS;
    // zero the ring once: the zero row (p + 2) is never written afterwards
    for (int i = tid; i < nslots * se; i += kZThreads) ring[i] = 0.0;
    if (tid == 0) {
        sm.tile = (lds_double*)ring;
        sm.slot_elems = se;
        sm.nslots = nslots;
    }
    if (tid < kZMaxSlots) { sm.ready[tid] = 0; sm.freed[tid] = 0; }
    __syncthreads();
    if (wave >= 4 && wave < 4 + kZProd) {
        __builtin_amdgcn_s_setprio(1);              // producers ahead of the MFMA consumers
        if (NT == 2) zgram_produce_pairs<NT, MODE, ZS>(g, sm, lane, wave - 4);
        else zgram_produce<NT, MODE, ZS>(g, sm, lane, wave - 4);
        return;
    }
    if (wave == 12) {
        // VALU-bound and on every slot's critical path: ahead of the producers' VALU on SIMD 0
        __builtin_amdgcn_s_setprio(2);
        if constexpr (ZCfg<NT>::BORDER) zgram_border_any<NT>(g, sm, lane);
        return;
    }
    if (wave == 0) {
        zgram_consume<NT, 0>(g, sm, lane);
    } else if (wave == 1) {
        zgram_consume<NT, 1>(g, sm, lane);
    } else if (wave == 2) {
        if constexpr (ZCfg<NT>::NCW >= 3) zgram_consume<NT, 2>(g, sm, lane);
    } else if constexpr (ZCfg<NT>::NCW == 4) {
        zgram_consume<NT, 3>(g, sm, lane);
    }
}

// ---- fixed pairwise trees over partials ----------------------------------------------------
// Group g sums the leaves [g*per, min((g+1)*per, total)) (per <= 32) over the binary tree of
// strides 1, 2, 4, 8, 16 (v[i] += v[i+s] for i a multiple of 2s) -- the tree composes: a rank
// that owns an aligned power-of-two run of leaves computes one of its subtrees.
// final != 0: write the symmetric Gram out[g][p2][p2]; else the merged partial out[g][PE].
template <int NT>
__global__ __launch_bounds__(256) void tree_merge_kernel(const double* in, int64_t total, int per,
                                                         int final_out, int p2, double* out) {
    using Cf = ZCfg<NT>;
    constexpr ZPairs<NT> tab{};
    const int64_t gi = blockIdx.x;
    const int64_t l0 = gi * per;
    const int n = (int)(total - l0 < per ? total - l0 : per);
    const double* src = in + l0 * Cf::PE;
    for (int e = blockIdx.y * 256 + threadIdx.x; e < Cf::PE; e += 256 * gridDim.y) {
        double v[32];
#pragma unroll
        for (int b = 0; b < 32; ++b) v[b] = b < n ? src[(int64_t)b * Cf::PE + e] : 0.0;
#pragma unroll
        for (int s = 1; s < 32; s *= 2)
#pragma unroll
            for (int i = 0; i + s < 32; i += 2 * s)
                if (i + s < n) v[i] = v[i] + v[i + s];
        if (!final_out) {
            out[gi * Cf::PE + e] = v[0];
        } else {
            const int q = e >> 8, r = (e >> 6) & 3, lane = e & 63;
            const int row = tab.I[q] * 16 + (lane >> 4) + 4 * r;    // f64 MFMA C/D layout
            const int col = tab.J[q] * 16 + (lane & 15);
            if (row < p2 && col < p2) {
                double* G = out + gi * (int64_t)p2 * p2;
                G[row * p2 + col] = v[0];
                G[col * p2 + row] = v[0];
            }
        }
    }
}

// ---- z-score statistics -> {mu, 1/sigma} and the surviving assets ------------------------------
__global__ __launch_bounds__(256) void zstats_finalize_kernel(const double* mu, const double* sd,
                                                              int K, int64_t lda, double* zs,
                                                              int32_t* asset_ok) {
    const int64_t a = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (a >= lda) return;
    int ok = 1;
    for (int k = 0; k < K; ++k) {
        const double m = mu[(int64_t)k * lda + a], s = sd[(int64_t)k * lda + a];
        const double r = 1.0 / s;
        // NaN sigma fails s > 0.  A subnormal sigma (< 2^-1024, 1/sigma overflows) also drops the
        // asset: the reference's (x - mu) / sigma could stay finite there, the product form
        // cannot ("z = (x - mu) * (1/sigma)").
        const bool okk = __builtin_isfinite(m) && s > 0.0 && __builtin_isfinite(r);
        ok &= okk ? 1 : 0;
        double2 v;
        v.x = okk ? m : 0.0;
        v.y = okk ? r : 0.0;
        reinterpret_cast<double2*>(zs)[(int64_t)k * lda + a] = v;
    }
    double2 one;
    one.x = 0.0;
    one.y = 1.0;
    reinterpret_cast<double2*>(zs)[(int64_t)K * lda + a] = one;   // row K: y passes unchanged
    asset_ok[a] = ok;
}

__global__ __launch_bounds__(256) void row_bits_kernel(int64_t nch, int64_t lda, const uint64_t* a,
                                                       const uint64_t* b, const int32_t* asset_ok,
                                                       int64_t t0, int64_t t1, uint64_t* out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nch * lda) return;
    const int64_t c = i / lda, as = i - c * lda;
    u64 w = a[i];
    if (b) w &= b[i];
    if (asset_ok && !asset_ok[as]) w = 0;
    const int64_t d0 = c << 6;
    if (t0 > d0) w &= t0 - d0 >= 64 ? 0ull : (~0ull << (t0 - d0));
    if (t1 - d0 < 64) w &= t1 <= d0 ? 0ull : ((1ull << (t1 - d0)) - 1ull);
    out[i] = w;
}

// pred[t][a] = b0 + sum_j b_j z_j, j ascending, zero coefficients skipped; NaN where the row bit
// is clear.  One thread per cell, 4 dates x 64 assets per workgroup.  The workgroup first
// compacts the non-zero coefficients (ascending j, by ballot) into LDS, so a sparse Lasso costs
// only its support per cell -- the same additions in the same order as the plain loop.
constexpr int kPredMaxP = 128;
__global__ __launch_bounds__(256) void zpredict_kernel(const double* base, int64_t col_stride,
                                                       int64_t lda, int64_t t0, int64_t nt,
                                                       const int32_t* cols, int p,
                                                       const double* zs, const double* beta,
                                                       const uint64_t* bits, double* pred) {
    __shared__ int sj[kPredMaxP];
    __shared__ double sb[kPredMaxP];
    __shared__ int snnz;
    const int tid = threadIdx.x;
    if (tid < 64) {                                  // wave 0: j = tid, tid + 64
        int cnt = 0;
        for (int j0 = 0; j0 < p; j0 += 64) {
            const int j = j0 + tid;
            const double bj = j < p ? beta[1 + j] : 0.0;
            const u64 m = __ballot(bj != 0.0);
            if (bj != 0.0) {
                const int pos = cnt + __popcll(m & ((1ull << tid) - 1ull));
                sj[pos] = j;
                sb[pos] = bj;
            }
            cnt += __popcll(m);
        }
        if (tid == 0) snnz = cnt;
    }
    __syncthreads();
    const int nnz = snnz;
    const int64_t a = (int64_t)blockIdx.x * 64 + (tid & 63);
    const int64_t t = t0 + (int64_t)blockIdx.y * 4 + (tid >> 6);
    if (t >= t0 + nt) return;
    const bool use = (bits[(t >> 6) * lda + a] >> (t & 63)) & 1ull;
    double v = __builtin_nan("");
    if (use) {
        double s = beta[0];
        const double* cell = base + t * lda + a;
        for (int q = 0; q < nnz; ++q) {
            const int j = sj[q];
            const double2 m = reinterpret_cast<const double2*>(zs)[(int64_t)j * lda + a];
            const double z = (cell[(int64_t)cols[j] * col_stride] - m.x) * m.y;
            s = s + sb[q] * z;
        }
        v = s;
    }
    pred[t * lda + a] = v;
}

}  // namespace
}  // namespace afm

using namespace afm;

// tile shape of a p-regressor design: 2 tiles (p + 2 <= 32) or 7 (p + 2 <= 108)
static int zgram_nt(int p) { return p + 2 <= 32 ? 2 : 7; }

extern "C" int afm_zgram_part_bytes(int p) {
    return (int)sizeof(double) * (zgram_nt(p) == 2 ? ZCfg<2>::PE : ZCfg<7>::PE);
}

template <int NT, int MODE, bool ZS>
static int launch_zgram(afm_ctx* ctx, const ZGramArgs& g, int64_t nitems, int grid) {
    int64_t wg = grid > 0 ? grid : 256;                 // persistent: one workgroup per CU
    if (wg > nitems) wg = nitems;
    if (wg <= 0) return AFM_OK;
    const int slot_bytes = (int)sizeof(double) * (g.p + 4) * kZRS;
    int nslots = kZLds / slot_bytes;
    if (nslots > kZMaxSlots) nslots = kZMaxSlots;
    AFM_CHECK_ARG(nslots >= 2, "ring does not fit in LDS");
    AFM_HIP(afm_lds_opt_in(ctx, (const void*)zgram_kernel<NT, MODE, ZS>, kZLds));
    hipLaunchKernelGGL((zgram_kernel<NT, MODE, ZS>), dim3((unsigned)wg), dim3(kZThreads),
                       (size_t)nslots * slot_bytes, ctx->stream, g, nslots);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

static int zgram_common_checks(const double* base, const int32_t* cols, const double* zs,
                               const uint64_t* bits, double* part, int p, int64_t lda,
                               int64_t a_end, int64_t blk0, int64_t t0, int64_t nt) {
    AFM_CHECK_ARG(base && cols && bits && part, "null buffer");
    AFM_CHECK_ARG(p >= 1 && p + 2 <= ZCfg<7>::KMAX, "need 1 <= p <= 106");
    AFM_CHECK_ARG(lda > 0 && lda % 64 == 0 && a_end <= lda, "lda must be a multiple of 64 >= a_end");
    AFM_CHECK_ARG(blk0 >= 0 && blk0 % 64 == 0, "blk0 must be a multiple of 64");
    AFM_CHECK_ARG(t0 >= 0 && nt >= 0, "bad date range");
    AFM_CHECK_ARG((t0 + nt) * lda * 8 < (int64_t)1 << 32 && lda * 16 * 112 < (int64_t)1 << 32,
                  "plane too large for 32-bit offsets");
    return AFM_OK;
}

extern "C" int afm_zgram_f64(afm_ctx* ctx, const double* base, int64_t col_stride, int64_t lda,
                             const int32_t* cols, const int32_t* zcols, int p, int ycol,
                             const double* zs, int zid, const uint64_t* bits, int64_t t0,
                             int64_t nt, int nblk, int64_t blk0, int64_t blk_assets,
                             int64_t a_end, double* part, int grid) {
    AFM_CTX(ctx);
    const int rc = zgram_common_checks(base, cols, zs, bits, part, p, lda, a_end, blk0, t0, nt);
    if (rc) return rc;
    AFM_CHECK_ARG(nblk >= 1 && blk_assets > 0 && blk_assets % 64 == 0 && nt * nblk < (1ll << 31),
                  "blocks must be 64-aligned");
    if (nt == 0) return AFM_OK;
    // the two-tile shape (NT = 2) stages item pairs (zgram_produce_pairs): even slot counts
    const int even = (!zs || zgram_nt(p) == 2) ? 1 : 0;
    ZGramArgs g{base, col_stride, lda, cols, zcols, p, ycol, zid, zs, bits, t0, nt, 0, nblk, blk0,
                blk_assets, a_end, 0, 1, part, even};
    if (!zs) return launch_zgram<2, 0, false>(ctx, g, nt * nblk, grid);   // FM: raw columns
    return zgram_nt(p) == 2 ? launch_zgram<2, 0, true>(ctx, g, nt * nblk, grid)
                            : launch_zgram<7, 0, true>(ctx, g, nt * nblk, grid);
}

extern "C" int afm_zpool_f64(afm_ctx* ctx, const double* base, int64_t col_stride, int64_t lda,
                             const int32_t* cols, const int32_t* zcols, int p, int ycol,
                             const double* zs, int zid, const uint64_t* bits, int64_t t0,
                             int64_t nt, int64_t blk0, int nrb, int64_t a_end, int nchunk,
                             double* part, int grid) {
    AFM_CTX(ctx);
    const int rc = zgram_common_checks(base, cols, zs, bits, part, p, lda, a_end, blk0, t0, nt);
    if (rc) return rc;
    AFM_CHECK_ARG(nrb >= 0 && nchunk >= 1 && (int64_t)nrb * nchunk < (1ll << 31), "bad leaves");
    if (nrb == 0) return AFM_OK;
    ZGramArgs g{base, col_stride, lda, cols, zcols, p, ycol, zid, zs, bits, t0, nt, 1, 1, blk0,
                64, a_end, nrb, nchunk, part, zgram_nt(p) == 2 ? 1 : 0};
    AFM_CHECK_ARG(zs != nullptr, "afm_zpool_f64 needs zs");
    return zgram_nt(p) == 2 ? launch_zgram<2, 1, true>(ctx, g, (int64_t)nrb * nchunk, grid)
                            : launch_zgram<7, 1, true>(ctx, g, (int64_t)nrb * nchunk, grid);
}

extern "C" int afm_gram_tree_f64(afm_ctx* ctx, int p, const double* in, int64_t total, int per,
                                 int final_out, double* out) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(in && out, "null buffer");
    AFM_CHECK_ARG(per >= 1 && per <= 32 && total >= 0, "need 1 <= per <= 32");
    AFM_CHECK_ARG(p >= 1 && p + 2 <= ZCfg<7>::KMAX, "need 1 <= p <= 106");
    if (total == 0) return AFM_OK;
    const unsigned ng = (unsigned)((total + per - 1) / per);
    if (zgram_nt(p) == 2)
        hipLaunchKernelGGL(tree_merge_kernel<2>, dim3(ng, 1), dim3(256), 0, ctx->stream, in, total,
                           per, final_out, p + 2, out);
    else
        hipLaunchKernelGGL(tree_merge_kernel<7>, dim3(ng, 4), dim3(256), 0, ctx->stream, in, total,
                           per, final_out, p + 2, out);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_zstats_finalize_f64(afm_ctx* ctx, const double* mu, const double* sd, int K,
                                       int64_t lda, double* zs, int32_t* asset_ok) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(mu && sd && zs && asset_ok, "null buffer");
    AFM_CHECK_ARG(K >= 1 && lda > 0, "bad shape");
    hipLaunchKernelGGL(zstats_finalize_kernel, dim3((unsigned)((lda + 255) / 256)), dim3(256), 0,
                       ctx->stream, mu, sd, K, lda, zs, asset_ok);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_row_bits(afm_ctx* ctx, int64_t nch, int64_t lda, const uint64_t* a,
                            const uint64_t* b, const int32_t* asset_ok, int64_t t0, int64_t t1,
                            uint64_t* out) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(a && out && nch >= 0 && lda > 0, "bad arguments");
    const int64_t n = nch * lda;
    if (n == 0) return AFM_OK;
    hipLaunchKernelGGL(row_bits_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       ctx->stream, nch, lda, a, b, asset_ok, t0, t1, out);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

extern "C" int afm_zpredict_f64(afm_ctx* ctx, const double* base, int64_t col_stride, int64_t lda,
                                int64_t t0, int64_t nt, const int32_t* cols, int p,
                                const double* zs, const double* beta, const uint64_t* bits,
                                double* pred) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(base && cols && zs && beta && bits && pred, "null buffer");
    AFM_CHECK_ARG(lda % 64 == 0 && nt >= 0 && t0 >= 0 && p >= 0 && p <= kPredMaxP, "bad shape");
    if (nt == 0) return AFM_OK;
    dim3 grid((unsigned)(lda / 64), (unsigned)((nt + 3) / 4));
    hipLaunchKernelGGL(zpredict_kernel, grid, dim3(256), 0, ctx->stream, base, col_stride, lda, t0,
                       nt, cols, p, zs, beta, bits, pred);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

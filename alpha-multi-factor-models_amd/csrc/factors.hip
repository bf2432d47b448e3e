// Factor panel: the 98 output columns of No-talib.py:1-93 for a
// calendar-grid panel, bit-exact with pandas 2.3.3.
//
// Layout (include/afm.h): inputs [T][lda] fp64 date-major/asset-minor, presence bits
// [ceil(T/64)][lda] uint64, output planes [98][T][lda].
//
// Kernel design (MI355X):
//  * One workgroup = 64 assets (one per lane) x 16 waves.  Every wave walks the SAME 64 assets
//    through time; each wave owns a fixed, compile-time set of indicator "jobs" whose state
//    (Kahan sums, Welford moments, ewm weights, cumsums) lives in its registers for the whole
//    series.  pandas' rolling/ewm kernels are sequential recurrences whose rounding depends on
//    the full history (Kahan compensation is never reset), so bit-exactness requires exactly
//    this: a sequential scan per asset, parallel over assets x job groups.
//  * Windows are positional over each asset's PRESENT days (holes and listing gaps do not count,
//    No-talib.py:5-6).  A shared LDS ring holds the last 128 present observations of close and
//    volume per lane (128 KB), indexed by the lane's observation count; 128 >= 57 (ACCEL_56
//    lookback) + 64 (chunk) + 1.  Derived series (returns, volume change, vol*close, up-days)
//    are recomputed from the ring with the same IEEE ops pandas uses.
//  * Time advances in chunks of 64 calendar days = one presence word.  Per chunk: the 16 waves
//    write the chunk's close/volume (prefetched into registers during the previous chunk) into
//    the ring (4 days each), barrier, every wave scans the 64 days for its jobs and streams
//    its output columns as coalesced 512-B row stores, barrier.  Absent cells are not written.
//  * dropna bookkeeping: each wave ORs a per-lane "some output NaN at day s" bit into an LDS
//    word; after the chunk wave 0 stores nanfree = present & ~nanmask.
//  * -ffp-contract=off + IEEE div/sqrt: every value rounds exactly as numpy/pandas on x86-64.
//
// Algorithmic traffic per present asset-day: 32 B of inputs read + 98 x 8 B written = 816 B.
#include "afm_internal.h"

#pragma clang fp contract(off)

namespace afm {
namespace {

constexpr int kLanes = 64;
constexpr int kRing = 128;
constexpr int kChunk = 64;
constexpr int kWaves = 16;
constexpr int kLoadSteps = kChunk / kWaves;  // 4 days loaded into the ring per wave per chunk

typedef unsigned long long u64;
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
    u64 nanmask[kLanes];
    u64 badmask[kLanes];       // some factor non-finite (NaN or +-inf)
};

struct Args {
    int64_t T, lda, plane;     // plane = T * lda
    const GLB double* close;
    const GLB double* volume;
    const GLB uint64_t* vbits;
    GLB double* out;
    GLB uint64_t* nanfree;
    GLB uint64_t* finite;      // optional
};

// Per-lane view of one (asset, present day) step.
struct Step {
    const LDS Smem* sm;
    GLB double* out;
    int64_t plane, cell;
    int lane, p;               // p = index of this observation in the asset's series
    bool anynan, anybad;
    __device__ __forceinline__ double C(int q) const { return sm->c[q & (kRing - 1)][lane]; }
    __device__ __forceinline__ double V(int q) const { return sm->v[q & (kRing - 1)][lane]; }
    __device__ __forceinline__ void put(int col, double x) {
        out[col * plane + cell] = x;
        anynan |= (x != x);
        anybad |= !__builtin_isfinite(x);
    }
    // close.pct_change() at q, with the window kernels' inf -> NaN (_prep_values)
    __device__ __forceinline__ double ret(int q) const {
        return q >= 1 ? C(q) / C(q - 1) - 1 : qnan();
    }
    __device__ __forceinline__ double volchg(int q) const {
        return q >= 1 ? V(q) / V(q - 1) - 1 : qnan();
    }
};

// ---- pandas window kernels as register-resident recurrences -------------------------------
// roll_mean (pandas/_libs/window/aggregations.pyx): Kahan add/remove with separate
// compensations, same-value run rule, sign rules.  prev starts as NaN: equivalent to pandas'
// "prev = values[0], run = 0" start for every first value.
struct RollMean {
    double sum, cadd, crem, prev;
    int nobs, neg, same;
    __device__ __forceinline__ void init() {
        sum = cadd = crem = 0.0;
        prev = qnan();
        nobs = neg = same = 0;
    }
    __device__ __forceinline__ void add(double x) {
        if (x == x) {
            nobs++;
            double y = x - cadd, t = sum + y;
            cadd = t - sum - y;
            sum = t;
            neg += __builtin_signbit(x) ? 1 : 0;
            same = (x == prev) ? same + 1 : 1;
            prev = x;
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
    __device__ __forceinline__ double result(int minp) const {
        if (nobs >= minp && nobs > 0) {
            double r = sum / (double)nobs;
            if (same >= nobs) r = prev;
            else if (neg == 0 && r < 0) r = 0.0;
            else if (neg == nobs && r > 0) r = 0.0;
            return r;
        }
        return qnan();
    }
};

// roll_var, ddof = 1: Welford with Kahan-compensated mean; the remove runs before the add.
struct RollVar {
    double mean, ssq, nobs, cadd, crem, prev;
    int same;
    __device__ __forceinline__ void init() {
        mean = ssq = nobs = cadd = crem = 0.0;
        prev = qnan();
        same = 0;
    }
    __device__ __forceinline__ void add(double x) {
        if (!__builtin_isnan(x)) {
            nobs = nobs + 1;
            same = (x == prev) ? same + 1 : 1;
            prev = x;
            double pm = mean - cadd, y = x - cadd, t = y - mean;
            cadd = t + mean - y;
            mean = (nobs != 0) ? mean + t / nobs : 0.0;
            ssq = ssq + (x - pm) * (x - mean);
        }
    }
    __device__ __forceinline__ void remove(double x) {
        if (!__builtin_isnan(x)) {
            nobs = nobs - 1;
            if (nobs != 0) {
                double pm = mean - crem, y = x - crem, t = y - mean;
                crem = t + mean - y;
                mean = mean - t / nobs;
                ssq = ssq - (x - pm) * (x - mean);
            } else {
                mean = 0.0;
                ssq = 0.0;
            }
        }
    }
    __device__ __forceinline__ double result(int minp) const {
        if (nobs >= (double)minp && nobs > 1.0)
            return (nobs == 1.0 || (double)same >= nobs) ? 0.0 : ssq / (nobs - 1.0);
        return qnan();
    }
};

// ewm(adjust=False, ignore_na=False).mean(), minp = 1.  wtd starts NaN / old = 1, which
// reproduces pandas' special first element exactly.  pandas emits wtd once nobs >= 1; wtd is
// NaN exactly until the first observation, so the emitted value is wtd itself.
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
                    wtd = old * wtd + nw * cur;
                    wtd /= (old + nw);
                }
                old = 1.0;
            }
        } else if (obs) {
            wtd = cur;
        }
        return wtd;
    }
};

// alpha = 1 / (1 + com) exactly as pandas computes it (constant-folded in IEEE double)
template <int SPAN>
struct SpanC {
    static constexpr double com = (SPAN - 1) / 2.0;
    static constexpr double alpha = 1.0 / (1.0 + com);
    static constexpr double owf = 1.0 - alpha;
};
template <int COM>
struct ComC {
    static constexpr double alpha = 1.0 / (1.0 + (double)COM);
    static constexpr double owf = 1.0 - alpha;
};

// ---- jobs (one output group each; columns in No-talib.py order, see abi.cpp) --------------
template <int W>
struct Sma {  // No-talib.py:9-10
    RollMean m;
    __device__ void init() { m.init(); }
    __device__ void step(Step& s) {
        if (s.p >= W) m.remove(s.C(s.p - W));
        m.add(s.C(s.p));
        s.put((W - 6) / 4, m.result(W));
    }
};

template <int W>
struct Ema {  // No-talib.py:13-14
    Ewm e;
    __device__ void init() { e.init(); }
    __device__ void step(Step& s) {
        s.put(12 + (W - 6) / 4, e.step(s.C(s.p), SpanC<W>::owf, SpanC<W>::alpha));
    }
};

template <int W>
struct Vwma {  // No-talib.py:17-19
    RollMean mvc, mv;
    __device__ void init() { mvc.init(); mv.init(); }
    __device__ void step(Step& s) {
        if (s.p >= W) {
            int q = s.p - W;
            mvc.remove(pinf(s.V(q) * s.C(q)));
            mv.remove(s.V(q));
        }
        mvc.add(pinf(s.V(s.p) * s.C(s.p)));
        mv.add(s.V(s.p));
        s.put(24 + (W - 6) / 4, mvc.result(W) / mv.result(W));
    }
};

template <int W>
struct Bbands {  // No-talib.py:22-26
    RollMean m;
    RollVar v;
    __device__ void init() { m.init(); v.init(); }
    __device__ void step(Step& s) {
        if (s.p >= W) {
            double x = s.C(s.p - W);
            m.remove(x);
            v.remove(x);
        }
        double x = s.C(s.p);
        m.add(x);
        v.add(x);
        double ma = m.result(W), sd = zsqrt(v.result(W));
        const int col = 36 + 2 * ((W - 14) / 6);
        s.put(col, ma + (2 * sd));
        s.put(col + 1, ma - (2 * sd));
    }
};

template <int W>
struct MomAccelRocr {  // No-talib.py:35-44
    __device__ void init() {}
    __device__ void step(Step& s) {
        const int k = (W - 14) / 6;
        double c = s.C(s.p);
        double mom = qnan(), acc = qnan(), roc = qnan();
        if (s.p >= W) {
            double cw = s.C(s.p - W);
            mom = c - cw;
            roc = c / cw - 1;
            if (s.p >= W + 1) acc = mom - (s.C(s.p - 1) - s.C(s.p - 1 - W));
        }
        s.put(52 + k, mom);
        s.put(60 + k, acc);
        s.put(68 + k, roc);
    }
};

template <int SLOW>
struct Macd {  // No-talib.py:47-50
    Ewm fast, slow;
    __device__ void init() { fast.init(); slow.init(); }
    __device__ void step(Step& s) {
        double c = s.C(s.p);
        double f = fast.step(c, SpanC<12>::owf, SpanC<12>::alpha);
        double l = slow.step(c, SpanC<SLOW>::owf, SpanC<SLOW>::alpha);
        s.put(76 + (SLOW - 18) / 6, f - l);
    }
};

template <int I>
struct Rsi {  // No-talib.py:53-59
    Ewm up, dn;
    __device__ void init() { up.init(); dn.init(); }
    __device__ void step(Step& s) {
        double d = s.p >= 1 ? s.C(s.p) - s.C(s.p - 1) : qnan();
        bool nan = (d != d);
        double u = (nan || d >= 0) ? d : 0.0;          // delta.clip(lower=0)
        double w = -((nan || d <= 0) ? d : 0.0);       // -delta.clip(upper=0)
        double eu = up.step(u, ComC<I - 1>::owf, ComC<I - 1>::alpha);
        double ed = dn.step(w, ComC<I - 1>::owf, ComC<I - 1>::alpha);
        double rs = eu / ed;
        s.put(79 + (I - 8) / 6, 100 - (100 / (1 + rs)));
    }
};

struct PvtObvPsy {  // No-talib.py:62-69
    double pvt, obv;
    int ups;
    __device__ void init() { pvt = 0.0; obv = 0.0; ups = 0; }
    __device__ void step(Step& s) {
        const int p = s.p;
        double c = s.C(p), v = s.V(p);
        // PVT: nan-skipping cumsum of volume * pct_change
        double term = p >= 1 ? v * (c / s.C(p - 1) - 1) : qnan();
        if (term == term) pvt = pvt + term;
        s.put(82, term == term ? pvt : qnan());
        // OBV: diff <= 0 (incl. equal closes) -> -volume, else (incl. NaN diff) +volume
        double d = p >= 1 ? c - s.C(p - 1) : qnan();
        double o = v * ((d <= 0) ? -1.0 : 1.0);
        if (o == o) obv = obv + o;
        s.put(83, o == o ? obv : qnan());
        // PSY: rolling(14) count of up-days / 14 * 100 (0/1 sums are exact)
        ups += (p >= 1 && c > s.C(p - 1)) ? 1 : 0;
        if (p >= 14) {
            int q = p - 14;
            ups -= (q >= 1 && s.C(q) > s.C(q - 1)) ? 1 : 0;
        }
        s.put(84, p >= 13 ? (double)ups / 14 * 100 : qnan());
    }
};

template <int W, int COL>
struct RetSd {  // sd_W of close.pct_change() (No-talib.py:72-74)
    RollVar v;
    __device__ void init() { v.init(); }
    __device__ double step(Step& s) {
        if (s.p >= W) v.remove(pinf(s.ret(s.p - W)));
        v.add(pinf(s.ret(s.p)));
        double r = zsqrt(v.result(W));
        s.put(COL, r);
        return r;
    }
};

struct RetSd3 {
    RetSd<3, 85> a;
    __device__ void init() { a.init(); }
    __device__ void step(Step& s) { a.step(s); }
};

struct RetSd5x15 {  // sd_5, sd_15, sd5_15
    RetSd<5, 86> a;
    RetSd<15, 87> b;
    __device__ void init() { a.init(); b.init(); }
    __device__ void step(Step& s) {
        double x = a.step(s), y = b.step(s);
        s.put(88, x / y);
    }
};

template <int W, int COL>
struct VolSd {  // volsd_W (No-talib.py:79-80)
    RollVar v;
    __device__ void init() { v.init(); }
    __device__ double step(Step& s) {
        if (s.p >= W) v.remove(pinf(s.V(s.p - W)));
        v.add(pinf(s.V(s.p)));
        double r = zsqrt(v.result(W));
        s.put(COL, r);
        return r;
    }
};

struct VolSd3 {
    VolSd<3, 89> a;
    __device__ void init() { a.init(); }
    __device__ void step(Step& s) { a.step(s); }
};

struct VolSd5x15 {
    VolSd<5, 90> a;
    VolSd<15, 91> b;
    __device__ void init() { a.init(); b.init(); }
    __device__ void step(Step& s) {
        double x = a.step(s), y = b.step(s);
        s.put(92, x / y);
    }
};

// ret.rolling(W).corr(vol_change) (No-talib.py:85-87; pandas Rolling.corr on prep_binary'd
// inputs).  WITH_VC also emits the vol_change column.
template <int W, bool WITH_VC>
struct Corr {
    RollMean mxy, mx, my;
    RollVar vx, vy;
    int cnt;
    __device__ void init() {
        mxy.init(); mx.init(); my.init(); vx.init(); vy.init();
        cnt = 0;
    }
    __device__ __forceinline__ static void xy(const Step& s, int q, double& X, double& Y) {
        double r = s.ret(q), g = s.volchg(q);
        X = pinf(r + 0 * g);
        Y = pinf(g + 0 * r);
    }
    __device__ void step(Step& s) {
        double X, Y;
        if (s.p >= W) {
            xy(s, s.p - W, X, Y);
            mxy.remove(X * Y);
            mx.remove(X);
            my.remove(Y);
            vx.remove(X);
            vy.remove(Y);
            double t = X + Y;
            cnt -= (t == t) ? 1 : 0;
        }
        xy(s, s.p, X, Y);
        mxy.add(X * Y);
        mx.add(X);
        my.add(Y);
        vx.add(X);
        vy.add(Y);
        double t = X + Y;
        cnt += (t == t) ? 1 : 0;
        double c = (double)cnt;
        double num = (mxy.result(W) - mx.result(W) * my.result(W)) * (c / (c - 1));
        double den = __builtin_sqrt(vx.result(W) * vy.result(W));
        s.put(94 + (W == 15 ? 1 : 0), num / den);
        if (WITH_VC) s.put(93, s.volchg(s.p));
    }
};

// ---- job packs ------------------------------------------------------------------------------
template <class... J>
struct Pack;
template <>
struct Pack<> {
    __device__ void init() {}
    __device__ void step(Step&) {}
};
template <class H, class... R>
struct Pack<H, R...> {
    H h;
    Pack<R...> r;
    __device__ void init() { h.init(); r.init(); }
    __device__ void step(Step& s) { h.step(s); r.step(s); }
};

// Static job partition over the 16 waves (roughly equal fp64 work per wave).
using W0 = Pack<Corr<5, true>>;
using W1 = Pack<Corr<15, false>>;
using W2 = Pack<Vwma<6>, Vwma<10>, Vwma<14>>;
using W3 = Pack<Vwma<18>, Vwma<22>, Vwma<26>>;
using W4 = Pack<Vwma<30>, Vwma<34>, Vwma<38>>;
using W5 = Pack<Vwma<42>, Vwma<46>, Vwma<50>>;
using W6 = Pack<Bbands<14>, Bbands<20>, MomAccelRocr<14>, MomAccelRocr<20>>;
using W7 = Pack<Bbands<26>, Bbands<32>, MomAccelRocr<26>, MomAccelRocr<32>>;
using W8 = Pack<Bbands<38>, Bbands<44>, MomAccelRocr<38>, MomAccelRocr<44>>;
using W9 = Pack<Bbands<50>, Bbands<56>, MomAccelRocr<50>, MomAccelRocr<56>>;
using W10 = Pack<Sma<6>, Sma<10>, Sma<14>, Sma<18>, Sma<22>, Sma<26>>;
using W11 = Pack<Sma<30>, Sma<34>, Sma<38>, Sma<42>, Sma<46>, Sma<50>>;
using W12 = Pack<RetSd3, RetSd5x15, PvtObvPsy>;
using W13 = Pack<VolSd3, VolSd5x15, Rsi<8>>;
using W14 = Pack<Ema<6>, Ema<10>, Ema<14>, Ema<18>, Ema<22>, Ema<26>, Ema<30>, Ema<34>,
                 Ema<38>, Ema<42>, Ema<46>, Ema<50>>;
using W15 = Pack<Macd<18>, Macd<24>, Macd<30>, Rsi<14>, Rsi<20>>;

template <class P>
__device__ __noinline__ void run_wave(const Args a, LDS Smem* smp, int wave, int lane) {
    LDS Smem& sm = *smp;
    const int64_t asset = (int64_t)blockIdx.x * kLanes + lane;
    const int nch = (int)((a.T + kChunk - 1) / kChunk);
    P jobs;
    jobs.init();
    int pos = 0;  // observations of this lane before the current chunk

    // prefetch chunk 0 (this wave's 4 days) and its presence word
    double pc[kLoadSteps], pv[kLoadSteps];
    u64 vb_next = a.vbits[asset];
#pragma unroll
    for (int j = 0; j < kLoadSteps; ++j) {
        int64_t t = wave * kLoadSteps + j;
        bool in = t < a.T;
        pc[j] = in ? a.close[t * a.lda + asset] : 0.0;
        pv[j] = in ? a.volume[t * a.lda + asset] : 0.0;
    }

    for (int ch = 0; ch < nch; ++ch) {
        const u64 vb = vb_next;
        // ring fill for this chunk (positions pos + rank of the day within the word)
#pragma unroll
        for (int j = 0; j < kLoadSteps; ++j) {
            const int s = wave * kLoadSteps + j;
            if ((vb >> s) & 1ull) {
                int q = pos + __popcll(vb & ((1ull << s) - 1ull));
                sm.c[q & (kRing - 1)][lane] = pc[j];
                sm.v[q & (kRing - 1)][lane] = pv[j];
            }
        }
        if (wave == 0) {
            sm.nanmask[lane] = 0ull;
            sm.badmask[lane] = 0ull;
        }
        // prefetch the next chunk while this one is scanned
        if (ch + 1 < nch) {
            vb_next = a.vbits[(int64_t)(ch + 1) * a.lda + asset];
#pragma unroll
            for (int j = 0; j < kLoadSteps; ++j) {
                int64_t t = (int64_t)(ch + 1) * kChunk + wave * kLoadSteps + j;
                bool in = t < a.T;
                pc[j] = in ? a.close[t * a.lda + asset] : 0.0;
                pv[j] = in ? a.volume[t * a.lda + asset] : 0.0;
            }
        }
        lds_barrier();

        const int64_t t0 = (int64_t)ch * kChunk;
        const int steps = (int)min((int64_t)kChunk, a.T - t0);
        u64 nb = 0ull, fb = 0ull;
        int p = pos;
        for (int s = 0; s < steps; ++s) {
            if ((vb >> s) & 1ull) {
                Step st;
                st.sm = smp;
                st.out = a.out;
                st.plane = a.plane;
                st.cell = (t0 + s) * a.lda + asset;
                st.lane = lane;
                st.p = p;
                st.anynan = false;
                st.anybad = false;
                jobs.step(st);
                if (st.anynan) nb |= 1ull << s;
                if (st.anybad) fb |= 1ull << s;
                ++p;
            }
        }
        if (nb) __atomic_fetch_or(&sm.nanmask[lane], nb, __ATOMIC_RELAXED);
        if (fb) __atomic_fetch_or(&sm.badmask[lane], fb, __ATOMIC_RELAXED);
        lds_barrier();
        if (wave == 0) {
            a.nanfree[(int64_t)ch * a.lda + asset] = vb & ~sm.nanmask[lane];
            if (a.finite) a.finite[(int64_t)ch * a.lda + asset] = vb & ~sm.badmask[lane];
        }
        pos = p;
    }
}

__global__ __launch_bounds__(kLanes * kWaves) void factor_panel_kernel(Args a) {
    __shared__ Smem sm_;
    LDS Smem* sm = (LDS Smem*)&sm_;
    const int lane = threadIdx.x & (kLanes - 1);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    switch (wave) {
        case 0: run_wave<W0>(a, sm, wave, lane); break;
        case 1: run_wave<W1>(a, sm, wave, lane); break;
        case 2: run_wave<W2>(a, sm, wave, lane); break;
        case 3: run_wave<W3>(a, sm, wave, lane); break;
        case 4: run_wave<W4>(a, sm, wave, lane); break;
        case 5: run_wave<W5>(a, sm, wave, lane); break;
        case 6: run_wave<W6>(a, sm, wave, lane); break;
        case 7: run_wave<W7>(a, sm, wave, lane); break;
        case 8: run_wave<W8>(a, sm, wave, lane); break;
        case 9: run_wave<W9>(a, sm, wave, lane); break;
        case 10: run_wave<W10>(a, sm, wave, lane); break;
        case 11: run_wave<W11>(a, sm, wave, lane); break;
        case 12: run_wave<W12>(a, sm, wave, lane); break;
        case 13: run_wave<W13>(a, sm, wave, lane); break;
        case 14: run_wave<W14>(a, sm, wave, lane); break;
        default: run_wave<W15>(a, sm, wave, lane); break;
    }
}

// target = excess_ret1d.shift(-1), tmr_ret1d = ret1d.shift(-1) (No-talib.py:90-91): the value of
// the asset's NEXT present day, NaN on its last one.  One thread per cell, next present day found
// from the presence words (ctz), rows read/written coalesced.
__global__ __launch_bounds__(256) void labels_kernel(int64_t T, int64_t lda, const double* excess,
                                                     const double* ret1d, const uint64_t* vbits,
                                                     double* target, double* tmr) {
    const int64_t a = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    const int64_t t = (int64_t)blockIdx.y * 4 + (threadIdx.x >> 6);
    if (t >= T) return;
    const int64_t nch = (T + 63) / 64;
    int64_t ch = t >> 6;
    const int s = (int)(t & 63);
    u64 w = vbits[ch * lda + a];
    if (!((w >> s) & 1ull)) return;
    u64 rest = (s == 63) ? 0ull : (w >> (s + 1)) << (s + 1);
    int64_t tn = -1;
    while (true) {
        if (rest) {
            tn = ch * 64 + __builtin_ctzll(rest);
            break;
        }
        if (++ch >= nch) break;
        rest = vbits[ch * lda + a];
    }
    const int64_t cell = t * lda + a;
    if (tn >= 0 && tn < T) {
        target[cell] = excess[tn * lda + a];
        tmr[cell] = ret1d[tn * lda + a];
    } else {
        target[cell] = __builtin_nan("");
        tmr[cell] = __builtin_nan("");
    }
}

}  // namespace
}  // namespace afm

extern "C" int afm_factors_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda,
                               const double* close, const double* volume, const double* ret1d,
                               const double* excess, const uint64_t* valid_bits, double* out,
                               uint64_t* nanfree_bits, uint64_t* finite_bits) {
    AFM_CTX(ctx);
    AFM_CHECK_ARG(T > 0 && A > 0, "T and A must be positive");
    AFM_CHECK_ARG(lda >= A && lda % 64 == 0, "lda must be a multiple of 64 and >= A");
    AFM_CHECK_ARG(close && volume && ret1d && excess && valid_bits && out && nanfree_bits,
                  "null buffer");
    AFM_CHECK_ARG(T <= (int64_t)1 << 31, "T too large");
    afm::Args a;
    a.T = T;
    a.lda = lda;
    a.plane = T * lda;
    a.close = (const GLB double*)close;
    a.volume = (const GLB double*)volume;
    a.vbits = (const GLB uint64_t*)valid_bits;
    a.out = (GLB double*)out;
    a.nanfree = (GLB uint64_t*)nanfree_bits;
    a.finite = (GLB uint64_t*)finite_bits;
    dim3 grid((unsigned)(lda / 64));
    hipLaunchKernelGGL(afm::factor_panel_kernel, grid, dim3(64 * 16), 0, ctx->stream, a);
    AFM_HIP(hipGetLastError());
    dim3 g2((unsigned)(lda / 64), (unsigned)((T + 3) / 4));
    hipLaunchKernelGGL(afm::labels_kernel, g2, dim3(256), 0, ctx->stream, T, lda, excess, ret1d,
                       valid_bits, out + 96 * a.plane, out + 97 * a.plane);
    AFM_HIP(hipGetLastError());
    return AFM_OK;
}

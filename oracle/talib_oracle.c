/* ORACLE -- test infrastructure only (never linked into the product).
 *
 * The TA-Lib columns of the reference's talib factor variant (KKT Yuliang Jiang.py:176-270,
 * SURVEY.md §8(f) rank 3), restated per series from TA-Lib 0.4's C core with
 * TA_COMPATIBILITY_DEFAULT and zero unstable periods, one function per TA-Lib routine, each
 * written in that routine's own loop structure (output index = input index; the first lookback
 * entries are NaN, as the Python wrapper returns them):
 *   ta_SMA.c  TA_INT_SMA    running total: add x[i], emit total / n, subtract x[i - n + 1]
 *   ta_EMA.c  TA_INT_EMA    seed = (0 + x[s-n+1] + ... + x[s]) / n at the start index s, then
 *                           prev = ((x - prev) * k) + prev, k = 2 / (n + 1)
 *   ta_BBANDS.c + TA_INT_stddev_using_precalc_ma   SMA middle, var = sumsq / n - middle^2,
 *                           sd = 0 when var < 1e-8, bands = middle +- sd * 2
 *   ta_MACD.c TA_INT_MACD   lookback = (signal - 1) + (slow - 1); both EMAs start at index
 *                           slow - 1 (TA_INT_EMA from there), macd = fast - slow
 *   ta_RSI.c                Wilder smoothing, 0 when |gain + loss| < 1e-8
 *   ta_OBV.c                starts at volume[0]; equal closes leave it unchanged
 * PVT here is volume * pct_change (no cumsum, KKT:229).  TA-Lib is absent from this container
 * and the reference ships no TA-Lib outputs, so these restatements are NOT pinned to TA-Lib
 * itself ("parity unpinned"); the HIP kernel (csrc/talib.hip) is checked against them.
 */
#include <math.h>
#include <stdint.h>

#define NC 68

static void sma(const double* x, int64_t n, int per, double* out, int64_t ld) {
    for (int64_t i = 0; i < n; ++i) out[i * ld] = NAN;
    if (n < per) return;
    double total = 0.0;
    int64_t i = 0, trailing = 0;
    while (i < per - 1) total += x[i++];
    do {
        total += x[i++];
        const double tmp = total;
        total -= x[trailing++];
        out[(i - 1) * ld] = tmp / per;
    } while (i < n);
}

static void ema_from(const double* x, int64_t n, int per, double k, int64_t start, double* buf) {
    /* TA_INT_EMA(startIdx = start): buf[i] for i >= start */
    int64_t today = start - (per - 1);
    double t = 0.0;
    for (int c = per; c-- > 0;) t += x[today++];
    double prev = t / per;
    while (today <= start) prev = ((x[today++] - prev) * k) + prev;
    buf[start] = prev;
    while (today < n) {
        prev = ((x[today] - prev) * k) + prev;
        buf[today++] = prev;
    }
}

static void ema(const double* x, int64_t n, int per, double* out, int64_t ld, double* buf) {
    for (int64_t i = 0; i < n; ++i) out[i * ld] = NAN;
    if (n < per) return;
    ema_from(x, n, per, 2.0 / (double)(per + 1), per - 1, buf);
    for (int64_t i = per - 1; i < n; ++i) out[i * ld] = buf[i];
}

static void bbands(const double* x, int64_t n, int per, double* up, double* mid, double* lo,
                   int64_t ld, double* mbuf) {
    for (int64_t i = 0; i < n; ++i) up[i * ld] = mid[i * ld] = lo[i * ld] = NAN;
    if (n < per) return;
    sma(x, n, per, mbuf, 1);
    int64_t start_sum = 0, end_sum = per - 1;
    double total2 = 0.0;
    for (int64_t i = start_sum; i < end_sum; ++i) total2 += x[i] * x[i];
    for (int64_t o = per - 1; o < n; ++o, ++start_sum, ++end_sum) {
        double t = x[end_sum];
        t *= t;
        total2 += t;
        double mv2 = total2 / per;
        t = x[start_sum];
        t *= t;
        total2 -= t;
        t = mbuf[o];
        t *= t;
        mv2 -= t;
        const double sd = (mv2 < 0.00000001) ? 0.0 : sqrt(mv2);
        const double d = sd * 2.0;
        up[o * ld] = mbuf[o] + d;
        mid[o * ld] = mbuf[o];
        lo[o * ld] = mbuf[o] - d;
    }
}

static void macd(const double* x, int64_t n, int fast, int slow, int signal, double* out,
                 int64_t ld, double* fb, double* sb) {
    for (int64_t i = 0; i < n; ++i) out[i * ld] = NAN;
    const int64_t look = (signal - 1) + (slow - 1);
    if (n <= look) return;
    const int64_t s = look - (signal - 1);
    ema_from(x, n, slow, 2.0 / (double)(slow + 1), s, sb);
    ema_from(x, n, fast, 2.0 / (double)(fast + 1), s, fb);
    for (int64_t i = look; i < n; ++i) out[i * ld] = fb[i] - sb[i];
}

static void rsi(const double* x, int64_t n, int per, double* out, int64_t ld) {
    for (int64_t i = 0; i < n; ++i) out[i * ld] = NAN;
    if (n <= per) return;
    int64_t today = 0;
    double prev_v = x[today], gain = 0.0, loss = 0.0;
    today++;
    for (int i = per; i > 0; i--) {
        const double v = x[today++];
        const double d = v - prev_v;
        prev_v = v;
        if (d < 0) loss -= d; else gain += d;
    }
    loss /= per;
    gain /= per;
    double s = gain + loss;
    out[per * ld] = (-0.00000001 < s && s < 0.00000001) ? 0.0 : 100.0 * (gain / s);
    while (today < n) {
        const double v = x[today];
        const double d = v - prev_v;
        prev_v = v;
        loss *= (per - 1);
        gain *= (per - 1);
        if (d < 0) loss -= d; else gain += d;
        loss /= per;
        gain /= per;
        s = gain + loss;
        out[today * ld] = (-0.00000001 < s && s < 0.00000001) ? 0.0 : 100.0 * (gain / s);
        today++;
    }
}

static void obv(const double* c, const double* v, int64_t n, double* out, int64_t ld) {
    if (n == 0) return;
    double o = v[0], prev = c[0];
    for (int64_t i = 0; i < n; ++i) {
        const double t = c[i];
        if (t > prev) o += v[i];
        else if (t < prev) o -= v[i];
        out[i * ld] = o;
        prev = t;
    }
}

/* One security's observations (close, volume) -> out [n][68] in the kernel's column order:
 * SMA 0-11, EMA 12-23, VSMA 24-35, BBANDS (upper, middle, lower) 36-59, MACD 60-62,
 * RSI 63-65, PVT 66, OBV 67.  work: 4 n doubles. */
void oracle_talib_series(int64_t n, const double* c, const double* v, double* out, double* work) {
    double* vc = work;
    double* b1 = work + n;
    double* b2 = work + 2 * n;
    for (int64_t i = 0; i < n; ++i) vc[i] = v[i] * c[i];
    for (int j = 0; j < 12; ++j) {
        const int per = 6 + 4 * j;
        sma(c, n, per, out + j, NC);
        ema(c, n, per, out + 12 + j, NC, b1);
        sma(vc, n, per, out + 24 + j, NC);
    }
    for (int j = 0; j < 8; ++j)
        bbands(c, n, 14 + 6 * j, out + 36 + 3 * j, out + 37 + 3 * j, out + 38 + 3 * j, NC, b1);
    for (int j = 0; j < 3; ++j) macd(c, n, 12, 18 + 6 * j, 9, out + 60 + j, NC, b1, b2);
    for (int j = 0; j < 3; ++j) rsi(c, n, 8 + 6 * j, out + 63 + j, NC);
    for (int64_t i = 0; i < n; ++i) out[i * NC + 66] = i >= 1 ? v[i] * (c[i] / c[i - 1] - 1) : NAN;
    obv(c, v, n, out + 67, NC);
}

int oracle_talib_panel(int64_t n_series, const int64_t* offsets, const double* c, const double* v,
                       double* out, double* work) {
    for (int64_t s = 0; s < n_series; ++s) {
        const int64_t o = offsets[s], n = offsets[s + 1] - o;
        oracle_talib_series(n, c + o, v + o, out + o * NC, work);
    }
    return 0;
}

/* ORACLE -- test infrastructure only (see factors_oracle.c header).
 *
 * Plain-C restatements of the per-date (cross-sectional) arithmetic the reference reaches through
 * pandas/numpy in "KKT Yuliang Jiang.py":
 *   - numpy pairwise summation (np.add.reduce on a contiguous float64 vector), used by
 *     Series.mean in the per-date demean (KKT:315-318) and the IR mean/std (KKT:353);
 *   - pandas libalgos.nancorr (Welford) for one column pair, used per date by
 *     DataFrame.corr('pearson') (KKT:344-345);
 *   - pandas libgroupby.group_mean (Kahan) used by groupby(...).mean() (KKT:331).
 * Pinned against tests/golden/analyzer_*.npz by tests/test_oracle_golden.py.
 */
#include <math.h>
#include <stdint.h>

/* numpy/_core/src/umath/loops_utils.h.src pairwise_sum (PW_BLOCKSIZE 128, 8-way unroll) */
static double pairwise(const double* a, int64_t n) {
    if (n < 8) {
        double res = 0.;
        for (int64_t i = 0; i < n; ++i) res += a[i];
        return res;
    } else if (n <= 128) {
        double r[8];
        for (int k = 0; k < 8; ++k) r[k] = a[k];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int k = 0; k < 8; ++k) r[k] += a[i + k];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return pairwise(a, n2) + pairwise(a + n2, n - n2);
    }
}

/* np.add.reduce on a contiguous float64 vector: the identity 0.0, then the pairwise sums of the
 * consecutive 8192-element buffers of the ufunc's buffered reduction (NPY_BUFSIZE) added one by
 * one -- a vector over 8192 elements is NOT one pairwise tree (tests/test_oracle_golden.py checks
 * this against numpy itself, up to 40,000 elements) */
double oracle_np_sum(int64_t n, const double* a) {
    double res = 0.0;
    for (int64_t i = 0; i < n; i += 8192) res += pairwise(a + i, n - i < 8192 ? n - i : 8192);
    return res;
}

/* nancorr for one pair (xi = the LATER column, yi = the earlier one), minp = 1 */
double oracle_nancorr_pair(int64_t n, const double* vxcol, const double* vycol) {
    int64_t nobs = 0;
    double ssqdmx = 0, ssqdmy = 0, covxy = 0, meanx = 0, meany = 0;
    for (int64_t i = 0; i < n; ++i) {
        double vx = vxcol[i], vy = vycol[i];
        if (isfinite(vx) && isfinite(vy)) {
            nobs += 1;
            double dx = vx - meanx, dy = vy - meany;
            meanx += 1. / nobs * dx;
            meany += 1. / nobs * dy;
            ssqdmx += (vx - meanx) * dx;
            ssqdmy += (vy - meany) * dy;
            covxy += (vx - meanx) * dy;
        }
    }
    if (nobs < 1) return NAN;
    double divisor = sqrt(ssqdmx * ssqdmy);
    /* pandas 2.3.3 returns covxy / divisor unclipped (|r| may exceed 1 by an ulp) */
    if (divisor != 0) return covxy / divisor;
    return NAN;
}

/* per-group nancorr over CSR groups */
void oracle_group_corr(int64_t n_groups, const int64_t* off, const double* vx, const double* vy,
                       double* out) {
    for (int64_t g = 0; g < n_groups; ++g)
        out[g] = oracle_nancorr_pair(off[g + 1] - off[g], vx + off[g], vy + off[g]);
}

/* group_mean with Kahan, rows visited in the given order; labels in [0, n_labels) or -1 */
void oracle_group_mean(int64_t n, const int64_t* labels, const double* v, int64_t n_labels,
                       double* sum, double* comp, int64_t* nobs, double* out) {
    for (int64_t k = 0; k < n_labels; ++k) { sum[k] = 0; comp[k] = 0; nobs[k] = 0; }
    for (int64_t i = 0; i < n; ++i) {
        int64_t lab = labels[i];
        if (lab < 0) continue;
        double val = v[i];
        if (val == val) {
            nobs[lab] += 1;
            double y = val - comp[lab];
            double t = sum[lab] + y;
            comp[lab] = t - sum[lab] - y;
            if (comp[lab] != comp[lab]) comp[lab] = 0;
            sum[lab] = t;
        }
    }
    for (int64_t k = 0; k < n_labels; ++k) out[k] = nobs[k] == 0 ? NAN : sum[k] / (double)nobs[k];
}

/* libgroupby.group_var (Welford, no Kahan), ddof=1, name="std" -> sqrt; K columns row-major */
void oracle_group_std(int64_t n, int64_t K, const int64_t* labels, const double* v, int64_t n_labels,
                      double* mean, int64_t* nobs, double* out) {
    for (int64_t k = 0; k < n_labels * K; ++k) { mean[k] = 0; nobs[k] = 0; out[k] = 0; }
    for (int64_t i = 0; i < n; ++i) {
        int64_t lab = labels[i];
        if (lab < 0) continue;
        for (int64_t j = 0; j < K; ++j) {
            double val = v[i * K + j];
            if (val == val) {
                int64_t q = lab * K + j;
                nobs[q] += 1;
                double old = mean[q];
                mean[q] += (val - old) / (double)nobs[q];
                out[q] += (val - mean[q]) * (val - old);
            }
        }
    }
    for (int64_t q = 0; q < n_labels * K; ++q) {
        double ct = (double)nobs[q];
        out[q] = (ct <= 1) ? NAN : sqrt(out[q] / (ct - 1));
    }
}

/* group_mean (Kahan), K columns row-major */
void oracle_group_mean2(int64_t n, int64_t K, const int64_t* labels, const double* v,
                        int64_t n_labels, double* sum, double* comp, int64_t* nobs, double* out) {
    for (int64_t k = 0; k < n_labels * K; ++k) { sum[k] = 0; comp[k] = 0; nobs[k] = 0; }
    for (int64_t i = 0; i < n; ++i) {
        int64_t lab = labels[i];
        if (lab < 0) continue;
        for (int64_t j = 0; j < K; ++j) {
            double val = v[i * K + j];
            if (val == val) {
                int64_t q = lab * K + j;
                nobs[q] += 1;
                double y = val - comp[q];
                double t = sum[q] + y;
                comp[q] = t - sum[q] - y;
                if (comp[q] != comp[q]) comp[q] = 0;
                sum[q] = t;
            }
        }
    }
    for (int64_t q = 0; q < n_labels * K; ++q) out[q] = nobs[q] == 0 ? NAN : sum[q] / (double)nobs[q];
}

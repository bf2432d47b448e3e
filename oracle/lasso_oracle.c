/* ORACLE -- test infrastructure only (never linked into the product).
 *
 * Lasso by cyclic coordinate descent on the centered Gram: the
 * reference fits sklearn's Lasso(alpha=2e-4, max_iter=10000) on the pooled train+valid design
 * (KKT Yuliang Jiang.py:605-607).  sklearn 1.7.2's ElasticNet.fit (l1_ratio = 1) centers X and
 * y, then minimises 0.5 ||y - X w||^2 + alpha n ||w||_1 by coordinate descent
 * (linear_model/_cd_fast.pyx).  This file restates its Gram variant,
 * enet_coordinate_descent_gram (Q = X'X, q = X'y, H = Q w kept up to date by two axpys per
 * coordinate), with the same coordinate update, the same stopping rule
 * (w_max == 0 or d_w_max / w_max < tol or last iteration -> duality gap < tol * y'y) and the same
 * gap formula; BLAS axpy is restated as a fused multiply-add per element and BLAS dot / asum as
 * sequential sums in feature order, which is also exactly what the HIP kernel does
 * (csrc/lasso.hip), so GPU == oracle bit for bit.  Against sklearn itself (residual-form CD on
 * X, BLAS reductions) the solutions agree to the solver tolerance; tests/golden holds sklearn
 * fits at tol 1e-4 and 1e-12 made in this container (tests/golden/make_lasso_golden.py).
 */
#include <math.h>
#include <stdint.h>

static double fsign(double f) { return f == 0.0 ? 0.0 : (f > 0.0 ? 1.0 : -1.0); }

/* Q [p][p] row-major, q [p], ynorm2 = y'y (all centered).  w [p] in/out (start value), info out:
 * [gap, tol * y'y, n_iter].  alpha here is the l1 weight of the unscaled objective (alpha * n). */
int oracle_lasso_gram(int p, const double* Q, const double* q, double ynorm2, double alpha,
                      double beta, int max_iter, double tol, int positive, double* w, double* H,
                      double* info) {
    double gap = tol + 1.0;
    const double d_w_tol = tol;
    tol = tol * ynorm2;
    for (int j = 0; j < p; ++j) {                       /* H = Q w (sequential rows) */
        double s = 0.0;
        for (int k = 0; k < p; ++k) s = s + Q[j * p + k] * w[k];
        H[j] = s;
    }
    int n_iter = 0;
    for (n_iter = 0; n_iter < max_iter; ++n_iter) {
        double w_max = 0.0, d_w_max = 0.0;
        for (int ii = 0; ii < p; ++ii) {
            const double qii = Q[ii * p + ii];
            if (qii == 0.0) continue;
            const double w_ii = w[ii];
            if (w_ii != 0.0)
                for (int j = 0; j < p; ++j) H[j] = fma(-w_ii, Q[ii * p + j], H[j]);
            const double tmp = q[ii] - H[ii];
            double wn;
            if (positive && tmp < 0) wn = 0.0;
            else wn = fsign(tmp) * fmax(fabs(tmp) - alpha, 0.0) / (qii + beta);
            w[ii] = wn;
            if (wn != 0.0)
                for (int j = 0; j < p; ++j) H[j] = fma(wn, Q[ii * p + j], H[j]);
            const double d_w_ii = fabs(wn - w_ii);
            if (d_w_ii > d_w_max) d_w_max = d_w_ii;
            if (fabs(wn) > w_max) w_max = fabs(wn);
        }
        if (w_max == 0.0 || d_w_max / w_max < d_w_tol || n_iter == max_iter - 1) {
            double q_dot_w = 0.0, wh = 0.0, w_norm2 = 0.0, asum = 0.0, dual = 0.0;
            for (int j = 0; j < p; ++j) {
                q_dot_w = q_dot_w + w[j] * q[j];
                const double xta = q[j] - H[j] - beta * w[j];
                const double a = positive ? xta : fabs(xta);
                if (j == 0 || a > dual) dual = a;
                wh = wh + w[j] * H[j];
                w_norm2 = w_norm2 + w[j] * w[j];
                asum = asum + fabs(w[j]);
            }
            const double r_norm2 = ynorm2 + wh - 2.0 * q_dot_w;
            double cst;
            if (dual > alpha) {
                cst = alpha / dual;
                const double a_norm2 = r_norm2 * (cst * cst);
                gap = 0.5 * (r_norm2 + a_norm2);
            } else {
                cst = 1.0;
                gap = r_norm2;
            }
            gap = gap + (alpha * asum - cst * ynorm2 + cst * q_dot_w +
                         0.5 * beta * (1 + cst * cst) * w_norm2);
            if (gap < tol) break;
        }
    }
    info[0] = gap;
    info[1] = tol;
    info[2] = (double)(n_iter < max_iter ? n_iter + 1 : max_iter);
    return 0;
}

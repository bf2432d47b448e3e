"""Golden vectors for the Lasso row: the reference calls scikit-learn's
``Lasso(alpha=2e-4, max_iter=10000).fit(X, y)`` (KKT Yuliang Jiang.py:605-607); this script runs
that estimator (scikit-learn 1.7.2 in this container) on small synthetic designs shaped like the
reference's (correlated z-scored factors, a noisy next-day-return target) and stores inputs and
fitted outputs.  Run from the repo root: python tests/golden/make_lasso_golden.py"""
import os
import warnings

import numpy as np
from sklearn.linear_model import Lasso

HERE = os.path.dirname(os.path.abspath(__file__))


def design(seed, n, p):
    rng = np.random.default_rng(seed)
    F = rng.normal(size=(n, p // 2))
    X = np.concatenate([F, F @ rng.normal(size=(p // 2, p - p // 2)) * 0.5
                        + rng.normal(size=(n, p - p // 2))], axis=1)
    X = (X - X.mean(0)) / X.std(0) + rng.normal(size=p) * 0.1
    beta = rng.normal(size=p) * 3e-3 * (rng.random(p) < 0.5)
    y = X @ beta + rng.normal(size=n) * 0.02 + 1e-4
    return X, y


def main():
    cases = {"ref": (1, 3000, 16, dict(alpha=2e-4, max_iter=10000)),
             "sparse": (2, 2000, 12, dict(alpha=2e-3, max_iter=10000)),
             "positive": (3, 2000, 8, dict(alpha=5e-4, max_iter=10000, positive=True)),
             "capped": (4, 1500, 16, dict(alpha=1e-6, max_iter=3))}
    out = {}
    for name, (seed, n, p, kw) in cases.items():
        X, y = design(seed, n, p)
        out[f"{name}_X"], out[f"{name}_y"] = X, y
        for tol in (1e-4, 1e-12):
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                m = Lasso(tol=tol, **kw).fit(X, y)
            k = f"{name}_tol{int(-np.log10(tol))}"
            out[f"{k}_coef"] = m.coef_
            out[f"{k}_intercept"] = np.array(m.intercept_)
            out[f"{k}_n_iter"] = np.array(m.n_iter_)
            out[f"{k}_dual_gap"] = np.array(m.dual_gap_)
        out[f"{name}_params"] = np.array([kw["alpha"], kw["max_iter"], kw.get("positive", 0)])
    np.savez_compressed(os.path.join(HERE, "lasso_sklearn.npz"), **out)


if __name__ == "__main__":
    main()

"""ORACLE -- test infrastructure only (see oracle/__init__.py).

CPU restatement of the chain ``afm.pipeline.Pipeline.step()`` runs -- the notebook cells that
feed ``PortfolioManager`` in the reference:

* factors            No-talib.py:1-93 (oracle.factors_long, the C restatement pinned to the
                     reference's goldens); all_df = the NT:33 dropna rows
* split + z-score    KKT:424-458 (oracle.pipeline: inclusive .loc date slices, Index.difference
                     feature order incl. tmr_ret1d, train-window group mean/std, inf -> NaN, dropna)
* Lasso              KKT:605-612: scikit-learn ``Lasso(alpha=2e-4, max_iter=10000)`` itself (the
                     reference's own dependency, present here) on concat(train, valid) in the
                     reference's (date, id) row order; ``predict`` on the test rows
* portfolio          KKT:976-977: oracle.portfolio.run_portfolio (exact box-QP in place of SLSQP,
                     SURVEY F6), history = target on the z-score-surviving rows, rolling window
* analyzer           KKT:630-631: oracle.xs.analyze on the test predictions and df_test closes
* Fama-MacBeth       the north-star per-date OLS: numpy lstsq per date of the target
                     on the raw FM factor columns of the same rows, oracle.pipeline.fama_macbeth

Inputs are a synthetic ``Panel`` (afm.synthetic); outputs are long arrays in (date, id) order.
"""
from __future__ import annotations

import time

import numpy as np

from . import FACTOR_NAMES, factors_long
from . import pipeline as PL
from . import portfolio as PF
from . import xs as XS

TARGET = FACTOR_NAMES.index("target")
TMR = FACTOR_NAMES.index("tmr_ret1d")
FEATURES = sorted(n for n in FACTOR_NAMES if n != "target")


def run_chain(p, train_end="2015-12-31", valid_end="2016-12-31", *, alpha=2e-4, max_iter=10000,
              tol=1e-4, fm_features=(), top_n=10, window=252, lo=0.0, hi=0.1, rate=1e-4,
              portfolio=True, analyzer=True, fm=True, timings=None):
    """The chain on panel ``p``; returns a dict of long arrays (rows in (date, id) order)."""
    tm = timings if timings is not None else {}
    t0 = time.perf_counter()
    v = p.valid[:, :p.A]
    aa, tt = np.nonzero(v.T)                                  # (asset, date) order: NT:2
    off = np.r_[0, np.cumsum(v.sum(axis=0))].astype(np.int64)
    fac = factors_long(off, p.close[tt, aa], p.volume[tt, aa], p.ret1d[tt, aa], p.excess[tt, aa])
    tm["factors"] = time.perf_counter() - t0
    t1 = time.perf_counter()
    # all rows in (date, id) order (the reference's all_df after set_index().sort_index(), KKT:275)
    o = np.lexsort((aa, tt))
    tt, aa, fac = tt[o], aa[o], fac[o]
    alldf = ~np.isnan(fac).any(axis=1)                        # NT:33 (inputs carry no NaN)
    dates = p.dates[tt].astype("datetime64[ns]")
    tr, va, te = PL.split_masks(dates, train_end, valid_end)
    fi = [FACTOR_NAMES.index(n) for n in FEATURES]
    X = fac[:, fi]
    uid = np.arange(p.A)
    m_tr = alldf & tr
    mu, sd = PL.group_stats(aa[m_tr], X[m_tr], uid)
    Z, keep = PL.zscore(aa, X, uid, mu, sd)
    zr = alldf & keep                                          # rows of df_*_x (KKT:452-458)
    y = fac[:, TARGET]
    tm["zscore"] = time.perf_counter() - t1
    t2 = time.perf_counter()
    from sklearn.linear_model import Lasso
    fit_rows = np.r_[np.flatnonzero(zr & tr), np.flatnonzero(zr & va)]
    las = Lasso(alpha=alpha, max_iter=max_iter, tol=tol).fit(Z[fit_rows], y[fit_rows])
    tst = np.flatnonzero(zr & te)
    pred = las.predict(Z[tst])
    tm["lasso"] = time.perf_counter() - t2
    res = {"n_fit": len(fit_rows), "coef": las.coef_.copy(), "intercept": float(las.intercept_),
           "n_iter": int(las.n_iter_), "pred_t": tt[tst], "pred_a": aa[tst], "pred": pred,
           "mu": mu, "sd": sd, "zrows_t": tt[zr], "zrows_a": aa[zr]}
    if not portfolio:
        return res
    t3 = time.perf_counter()
    # PortfolioManager(lasso_predict, df_train_y, all_df) with the north-star rolling window:
    # history = target on every z-surviving row; "all" rows = every present row (tradable, close,
    # tmr lookups, and the calendar of the window)
    dint = p.dates.astype("datetime64[ns]").astype(np.int64)
    pr = PF.run_portfolio(dint[tt[tst]], aa[tst], pred, dint[tt[zr]], aa[zr], y[zr],
                          dint[tt], aa, p.tradable[tt, aa], p.close[tt, aa], fac[:, TMR],
                          trading_cost_rate=rate, top_n=top_n, window=window, lo=lo, hi=hi)
    res["portfolio"] = pr
    tm["portfolio"] = time.perf_counter() - t3
    if analyzer:
        t4 = time.perf_counter()
        px = np.flatnonzero(alldf & te)                       # df_test[['close_price']]
        res["analyzer"] = XS.analyze(dint[tt[tst]], aa[tst], pred, dint[tt[px]], aa[px],
                                     p.close[tt[px], aa[px]])
        tm["analyzer"] = time.perf_counter() - t4
    if fm and len(fm_features):
        t5 = time.perf_counter()
        fj = [FACTOR_NAMES.index(n) for n in fm_features]      # raw factor values
        rows = np.flatnonzero(zr)
        d, B, N = PL.xs_ols(tt[rows], fac[rows][:, fj], y[rows])
        res["fm_dates"], res["fm_beta"], res["fm_n"] = d, B, N
        tm["fm"] = time.perf_counter() - t5
    return res

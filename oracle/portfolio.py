"""ORACLE -- test infrastructure only (see oracle/__init__.py).

Restatement of ``PortfolioManager`` ("KKT Yuliang Jiang.py":795-970), rows K1-K4 of SURVEY.md
§8(a).

Weight solve (K2, ``KKT:811-833``): the reference minimises sqrt(w'Sw) with SLSQP, sum(w)=1,
0<=w<=0.1.  SLSQP's default ftol leaves ~1e-3 error whenever a bound is active, so it is not a
parity target; this oracle solves the same problem EXACTLY with a primal
active-set method on the KKT system [S_FF 1; 1' 0][w_F; lam] = [-S_FB w_B; b] (Cholesky +
Schur complement), which is what the GPU kernel implements.  Where the problem has a single
feasible point (n*hi == 1, the reference's default top_n=10) both return hi exactly, and the
reference goldens (tests/golden/portfolio_pipeline.npz) pin that path bit-for-bit.  Where it is
infeasible (n*hi < 1) SLSQP stops at w=hi (status 4); this oracle returns w=hi.

Selections (K3): ``nlargest``/``nsmallest`` ties follow Python ``set`` iteration order in the
reference (KKT:848,855) -- not reproducible; here ties break by ascending id.
"""
from __future__ import annotations

import numpy as np

from .xs import np_sum


def box_qp_weights(S: np.ndarray, lo: float = 0.0, hi: float = 0.1, max_iter: int = 0):
    """min w'Sw  s.t. sum(w) = 1, lo <= w <= hi  (exact primal active set).  Returns (w, it)."""
    S = np.asarray(S, dtype=np.float64)
    n = S.shape[0]
    if n == 0:
        return np.zeros(0), 0
    if n * hi <= 1.0:
        return np.full(n, hi), 0
    if n * lo >= 1.0:
        return np.full(n, lo), 0
    max_iter = max_iter or 4 * n + 8
    w = np.full(n, 1.0 / n)
    state = np.zeros(n, dtype=np.int8)          # 0 free, -1 at lo, +1 at hi
    it = 0
    lam = 0.0
    while it < max_iter:
        it += 1
        F = np.flatnonzero(state == 0)
        B = np.flatnonzero(state != 0)
        b = 1.0 - w[B].sum()
        if len(F) == 0:
            break
        SFF = S[np.ix_(F, F)]
        c = S[np.ix_(F, B)] @ w[B] if len(B) else np.zeros(len(F))
        L = np.linalg.cholesky(SFF)
        y1 = np.linalg.solve(L.T, np.linalg.solve(L, np.ones(len(F))))
        y2 = np.linalg.solve(L.T, np.linalg.solve(L, c))
        lam = -(b + y2.sum()) / y1.sum()
        x = -y2 - lam * y1
        if np.all(x >= lo) and np.all(x <= hi):
            w[F] = x
            g = S @ w + lam
            viol = np.where(state == -1, g, np.where(state == 1, -g, np.inf))
            j = int(np.argmin(viol))
            if viol[j] >= 0:
                break
            state[j] = 0
            continue
        p = x - w[F]
        alpha, jb, bound = 1.0, -1, 0
        for k, i in enumerate(F):
            if x[k] < lo and p[k] < 0:
                a = (lo - w[i]) / p[k]
                if a < alpha:
                    alpha, jb, bound = a, i, -1
            elif x[k] > hi and p[k] > 0:
                a = (hi - w[i]) / p[k]
                if a < alpha:
                    alpha, jb, bound = a, i, 1
        w[F] = w[F] + alpha * p
        if jb >= 0:
            w[jb] = lo if bound < 0 else hi
            state[jb] = bound
    return w, it


def pairwise_cov(R: np.ndarray) -> np.ndarray:
    """DataFrame.cov(): np.cov when NaN-free, else pandas nancorr(cov=True) (pairwise)."""
    R = np.asarray(R, dtype=np.float64)
    if np.isfinite(R).all():
        return np.atleast_2d(np.cov(R.T, ddof=1))
    n, k = R.shape
    out = np.full((k, k), np.nan)
    fin = np.isfinite(R)
    for xi in range(k):
        for yi in range(xi + 1):
            m = fin[:, xi] & fin[:, yi]
            vx, vy = R[m, xi], R[m, yi]
            nobs, mx, my, cov = 0, 0.0, 0.0, 0.0
            for a, bb in zip(vx.tolist(), vy.tolist()):
                nobs += 1
                dx, dy = a - mx, bb - my
                mx += 1.0 / nobs * dx
                my += 1.0 / nobs * dy
                cov += (a - mx) * dy
            if nobs >= 1 and nobs - 1.0 != 0:
                out[xi, yi] = out[yi, xi] = cov / (nobs - 1.0)
    return out


def select_books(ids: np.ndarray, vals: np.ndarray, tradable: np.ndarray, top_n: int):
    """KKT:847-856: tradable & predicted; top_n shrinks to n//2 on thin dates; long = nlargest
    (descending), short = nsmallest (ascending); ties by ascending id."""
    m = tradable
    ti, tv = ids[m], vals[m]
    n = len(ti)
    k = n // 2 if n < 2 * top_n else top_n
    o = np.lexsort((ti, -tv))
    long_ids = ti[o[:k]]
    o2 = np.lexsort((ti, tv))
    short_ids = ti[o2[:k]]
    return long_ids, short_ids


def book_history(hist_date, hist_id, hist_val, book, window: int | None = None, upto=None,
                 calendar=None):
    """KKT:858-859: history.swaplevel().loc[book].unstack().T -> [dates x book] with NaN holes.
    ``window``/``upto``/``calendar``: keep history dates in the ``window`` calendar dates that
    precede ``upto`` (the north-star rolling window); None reproduces the reference (the whole
    training window)."""
    m = np.isin(hist_id, book)
    missing = set(book.tolist()) - set(hist_id[m].tolist())
    if missing:
        raise KeyError(f"{sorted(missing)} not in history")
    d, i, v = hist_date[m], hist_id[m], hist_val[m]
    if window is not None:
        cal = np.asarray(calendar)
        j = int(np.searchsorted(cal, upto))
        first = cal[max(0, j - window)]
        k = (d >= first) & (d < upto)
        d, i, v = d[k], i[k], v[k]
    dates = np.unique(d)
    col = {x: j for j, x in enumerate(book.tolist())}
    R = np.full((len(dates), len(book)), np.nan)
    R[np.searchsorted(dates, d), [col[x] for x in i.tolist()]] = v
    return R


def _date_books(dt, pred_date, pred_id, pred, hist_date, hist_id, hist, akey, all_tradable,
                all_close, all_tmr, calendar, top_n, window, lo, hi):
    """The path-independent part of one rebalance date (KKT:844-877): books, weights, PnL sums."""
    m = pred_date == dt
    ids, vals = pred_id[m], pred[m]
    rows = np.array([akey.get((dt, i), -1) for i in ids.tolist()])
    trad = np.array([r >= 0 and bool(all_tradable[r]) for r in rows])
    L, S = select_books(ids, vals, trad, top_n)
    wl = box_qp_weights(pairwise_cov(book_history(hist_date, hist_id, hist, L, window, dt,
                                                  calendar)), lo, hi)[0]
    ws = box_qp_weights(pairwise_cov(book_history(hist_date, hist_id, hist, S, window, dt,
                                                  calendar)), lo, hi)[0]
    rl = np.array([all_tmr[akey[(dt, i)]] for i in L.tolist()])
    rs = np.array([all_tmr[akey[(dt, i)]] for i in S.tolist()])
    pl = np.array([all_close[akey[(dt, i)]] for i in L.tolist()])
    ps = np.array([all_close[akey[(dt, i)]] for i in S.tolist()])
    lsum, ssum = np_sum(np.nan_to_num(rl * wl)), np_sum(np.nan_to_num(rs * ws))
    den_l = 0
    for x in (wl * pl).tolist():                 # builtin sum(): 0 + x0 + x1 ...
        den_l = den_l + x
    den_s = 0
    for x in (ws * ps).tolist():
        den_s = den_s + x
    return dict(ids=ids, L=L, S=S, wl=wl, ws=ws, lsum=lsum, ssum=ssum, den_l=den_l, den_s=den_s)


def _value_recursion(seq, trading_cost_rate, v0=100000000.0):
    """KKT:864-892 over a sequence of per-date records (a date may repeat: bootstrap paths)."""
    V = [v0]
    turnovers, long_r, short_r = [], [], []
    cur = None                                   # (ids, positions) of the previous step
    for b in seq:
        ids = b["ids"]
        size = V[-1] / 2
        daily = (b["lsum"] - b["ssum"]) / 2
        long_r.append(b["lsum"])
        short_r.append(b["ssum"])
        newpos = np.full(len(ids), np.nan)
        idx = {x: j for j, x in enumerate(ids.tolist())}
        for x in b["L"].tolist():
            newpos[idx[x]] = size / b["den_l"]
        for x in b["S"].tolist():
            newpos[idx[x]] = -size / b["den_s"]
        if cur is None or np.all(np.isnan(cur[1])):
            to = 0.0
        else:                                    # (cur.fillna(0) - new.fillna(0)) on the union
            u = np.union1d(cur[0], ids)
            a = np.full(len(u), np.nan)
            bvec = np.full(len(u), np.nan)
            a[np.searchsorted(u, cur[0])] = np.nan_to_num(cur[1])
            bvec[np.searchsorted(u, ids)] = np.nan_to_num(newpos)
            dlt = np.abs(a - bvec)
            to = np_sum(np.where(np.isnan(dlt), 0.0, dlt)) / 2
        turnovers.append(to)
        cost = to * trading_cost_rate
        daily -= cost / V[-1]
        V.append(V[-1] * (1 + daily))
        cur = (ids, newpos)
    return {"value": np.array(V), "turnover": np.array(turnovers), "long_ret": np.array(long_r),
            "short_ret": np.array(short_r)}


def _all_books(pred_date, pred_id, pred, hist_date, hist_id, hist, all_date, all_id,
               all_tradable, all_close, all_tmr, top_n, window, lo, hi):
    akey = {(d, i): j for j, (d, i) in enumerate(zip(all_date.tolist(), all_id.tolist()))}
    udates = np.unique(pred_date)
    calendar = np.unique(np.concatenate([pred_date, hist_date, all_date]))
    recs = [_date_books(dt, pred_date, pred_id, pred, hist_date, hist_id, hist, akey,
                        all_tradable, all_close, all_tmr, calendar, top_n, window, lo, hi)
            for dt in udates]
    return udates, recs


def run_portfolio(pred_date, pred_id, pred, hist_date, hist_id, hist, all_date, all_id,
                  all_tradable, all_close, all_tmr, trading_cost_rate=1e-4, top_n=10,
                  window=None, lo=0.0, hi=0.1):
    """PortfolioManager.calculate_portfolio (KKT:842-892) with the exact weight solve."""
    udates, recs = _all_books(pred_date, pred_id, pred, hist_date, hist_id, hist, all_date,
                              all_id, all_tradable, all_close, all_tmr, top_n, window, lo, hi)
    res = _value_recursion(recs, trading_cost_rate)
    res["books"] = [x for b in recs for x in (b["L"], b["S"])]
    res["weights"] = [x for b in recs for x in (b["wl"], b["ws"])]
    res["dates"] = udates
    return res


def run_bootstrap(paths, pred_date, pred_id, pred, hist_date, hist_id, hist, all_date, all_id,
                  all_tradable, all_close, all_tmr, trading_cost_rate=1e-4, top_n=10,
                  window=None, lo=0.0, hi=0.1):
    """Bootstrap of the rebalance sequence (BASELINE config E): ``paths`` [npaths][steps] indices
    into the sorted unique prediction dates; every path re-runs the KKT:864-892 recursion over
    its steps (books per date are path-independent)."""
    _, recs = _all_books(pred_date, pred_id, pred, hist_date, hist_id, hist, all_date, all_id,
                         all_tradable, all_close, all_tmr, top_n, window, lo, hi)
    out = [_value_recursion([recs[j] for j in row], trading_cost_rate) for row in np.asarray(paths)]
    return {k: np.stack([o[k] for o in out]) for k in out[0]} if out else {}


def sharpe(V):
    """KKT:894-897: pct_change().dropna(); mean / std (ddof 1)."""
    from .xs import nanmean, nanstd
    V = np.asarray(V, dtype=np.float64)
    r = V[1:] / V[:-1] - 1
    return nanmean(r) / nanstd(r)


def annualized_return(V):
    """KKT:945-949."""
    total = V[-1] / V[0] - 1
    years = len(V) / 252
    return (1 + total) ** (1 / years) - 1


def max_drawdown(V):
    """KKT:951-955."""
    V = np.asarray(V, dtype=np.float64)
    rm = np.maximum.accumulate(V)
    return float(((rm - V) / rm).max())

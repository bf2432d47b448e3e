"""ORACLE -- test infrastructure only (see oracle/__init__.py).

Array restatement of ``AlphaSignalAnalyzer`` ("KKT Yuliang Jiang.py":280-375), rows A1-A4 of
SURVEY.md §8(a).  Inputs are long arrays in the reference's (date, id)-sorted row order:

* signal rows ``(sig_date, sig_id, sig_val)``  -- ``alpha_signal_df`` (KKT:281-283)
* price rows ``(px_date, px_id, px_close)``    -- ``price_data`` (KKT:291-293)

Outputs mirror the reference attributes (``ic_df``, ``ir_df``, ``layered_ret_dfs``,
``ls_ret_dfs``, ``port_ret_df``) as flat arrays.  Pinned against tests/golden/analyzer_*.npz.
"""
from __future__ import annotations

import numpy as np

from . import _p, lib

RETURN_TYPES = ("return_1", "return_2", "return_5")   # KKT:290
K_LAYERS = 10                                         # KKT:287
TOP_K = 10                                            # KKT:288


def np_sum(v: np.ndarray) -> float:
    v = np.ascontiguousarray(v, dtype=np.float64)
    return lib().oracle_np_sum(len(v), _p(v))


def nanmean(v: np.ndarray) -> float:
    """pandas nanops.nanmean on a NaN-free vector: pairwise sum / count."""
    return np_sum(v) / float(len(v)) if len(v) else np.nan


def nanstd(v: np.ndarray) -> float:
    """pandas nanops.nanstd, ddof=1, two-pass (sum((avg - x)**2) / (n - 1))."""
    n = len(v)
    if n <= 1:
        return np.nan
    avg = np_sum(v) / float(n)
    sqr = (avg - v) ** 2
    return float(np.sqrt(np_sum(sqr) / (float(n) - 1.0)))


def group_starts(keys: np.ndarray) -> np.ndarray:
    """CSR offsets of runs of equal consecutive keys."""
    if len(keys) == 0:
        return np.zeros(1, np.int64)
    s = np.flatnonzero(np.r_[True, keys[1:] != keys[:-1]])
    return np.r_[s, len(keys)].astype(np.int64)


def forward_returns(px_date, px_id, px_close, k: int) -> np.ndarray:
    """KKT:311: per id, positional ``close.pct_change(k).shift(-k)`` over the price rows."""
    order = np.lexsort((px_date, px_id))          # by id, then date
    c = px_close[order]
    i = px_id[order]
    r = np.full(len(c), np.nan)
    if len(c) > k:
        same = i[k:] == i[:-k]
        with np.errstate(all="ignore"):
            v = c[k:] / c[:-k] - 1
        r[:-k] = np.where(same, v, np.nan)
    out = np.empty_like(r)
    out[order] = r
    return out


def add_returns(sig_date, sig_id, sig_val, px_date, px_id, px_close):
    """KKT:308-320 -> (date, id, [factor, return_1, return_2, return_5]) rows."""
    date, ids = np.asarray(sig_date), np.asarray(sig_id)
    cols = [np.asarray(sig_val, dtype=np.float64)]
    pkey = {(d, i): j for j, (d, i) in enumerate(zip(px_date.tolist(), px_id.tolist()))}
    for rt in RETURN_TYPES:
        k = int(rt[-1])
        fr = forward_returns(px_date, px_id, px_close, k)
        fr = np.where(fr <= 1, fr, np.nan)                       # KKT:312
        idx = np.array([pkey.get((d, i), -1) for d, i in zip(date.tolist(), ids.tolist())],
                       dtype=np.int64)
        r = np.where(idx >= 0, fr[np.maximum(idx, 0)], np.nan)   # left merge (KKT:313)
        keep = ~np.isnan(r)
        for c in cols:
            keep &= ~np.isnan(c)
        date, ids = date[keep], ids[keep]
        cols = [c[keep] for c in cols] + [r[keep]]
        # per-date demean (KKT:315-318), rows in (date, original) order
        order = np.argsort(date, kind="stable")
        date, ids = date[order], ids[order]
        cols = [c[order] for c in cols]
        off = group_starts(date)
        x = cols[-1].copy()
        for g in range(len(off) - 1):
            s, e = off[g], off[g + 1]
            x[s:e] = x[s:e] - nanmean(x[s:e])
        cols[-1] = x
    return date, ids, np.stack(cols, axis=1)


def ic_series(date, vals):
    """KKT:342-349: per date, nancorr(return_k, factor) (return = the later column)."""
    off = group_starts(date)
    L = lib()
    out_d, out_t, out_ic = [], [], []
    f = np.ascontiguousarray(vals[:, 0])
    for g in range(len(off) - 1):
        s, e = off[g], off[g + 1]
        for k, rt in enumerate(RETURN_TYPES):
            r = np.ascontiguousarray(vals[s:e, 1 + k])
            ic = L.oracle_nancorr_pair(e - s, _p(r), _p(np.ascontiguousarray(f[s:e])))
            if not np.isnan(ic):                      # .stack() drops NaN
                out_d.append(date[s]); out_t.append(rt); out_ic.append(ic)
    return np.array(out_d), np.array(out_t), np.array(out_ic, dtype=np.float64)


def ir_table(ic_date, ic_type, ic):
    """KKT:351-354: per (year, Type): mean(IC) / std(IC)."""
    years = np.asarray(ic_date).astype("datetime64[ns]").astype("datetime64[Y]").astype(np.int64) + 1970
    res = []
    for y in sorted(set(years.tolist())):
        for rt in sorted(set(ic_type.tolist())):
            m = (years == y) & (ic_type == rt)
            if m.any():
                v = ic[m]
                res.append((y, rt, nanmean(v) / nanstd(v)))
    return (np.array([r[0] for r in res]), np.array([r[1] for r in res]),
            np.array([r[2] for r in res], dtype=np.float64))


def rank_first(v: np.ndarray, ascending: bool = True) -> np.ndarray:
    """groupby rank(method='first') within one group: 1..n, ties by row position."""
    order = np.argsort(v if ascending else -v, kind="stable")
    r = np.empty(len(v), dtype=np.float64)
    r[order] = np.arange(1, len(v) + 1, dtype=np.float64)
    return r


def layers(date, vals, k: int):
    """KKT:324-340 for return column ``k`` (1-based into vals)."""
    off = group_starts(date)
    nd = len(off) - 1
    lab = np.empty(len(date), dtype=np.int64)
    for g in range(nd):
        s, e = off[g], off[g + 1]
        pct = rank_first(vals[s:e, 0]) / float(e - s)
        layer = (pct * K_LAYERS).astype(np.int64) + 1
        layer[layer > K_LAYERS] = K_LAYERS
        lab[s:e] = g * K_LAYERS + (layer - 1)
    nl = nd * K_LAYERS
    sums, comp, out = np.zeros(nl), np.zeros(nl), np.zeros(nl)
    nobs = np.zeros(nl, dtype=np.int64)
    v = np.ascontiguousarray(vals[:, k])
    lib().oracle_group_mean(len(v), _p(lab), _p(v), nl, _p(sums), _p(comp), _p(nobs), _p(out))
    mean = np.where(nobs > 0, out, np.nan).reshape(nd, K_LAYERS)
    present = (nobs.reshape(nd, K_LAYERS) > 0).any(axis=0)
    cum = np.full_like(mean, np.nan)
    for j in range(K_LAYERS):                     # DataFrame.cumsum (skipna) per layer
        s = 0.0
        for i in range(nd):
            x = mean[i, j]
            if x == x:
                s = s + x
                cum[i, j] = s
    dates = date[off[:-1]]
    lay_layers = np.flatnonzero(present) + 1
    # layered_ret_dfs: stack() (row-major, NaN dropped)
    ld, ll, lv = [], [], []
    for i in range(nd):
        for l in lay_layers:
            x = cum[i, l - 1]
            if x == x:
                ld.append(dates[i]); ll.append(l); lv.append(x)
    # ls_ret_dfs: {5 - l + 1: cum[10 - l + 1] - cum[l]} for l = 1..5
    sd, sl, sv = [], [], []
    for i in range(nd):
        for l in range(1, K_LAYERS // 2 + 1):
            x = cum[i, K_LAYERS - l] - cum[i, l - 1]
            if x == x:
                sd.append(dates[i]); sl.append(K_LAYERS // 2 - l + 1); sv.append(x)
    return ((np.array(ld), np.array(ll, dtype=np.int64), np.array(lv, dtype=np.float64)),
            (np.array(sd), np.array(sl, dtype=np.int64), np.array(sv, dtype=np.float64)))


# string-rank pivot column order (KKT:362-365): '1.0','10.0','2.0',...,'9.0'
_PIVOT_ORDER = sorted([f"{float(r)}" for r in range(1, TOP_K + 1)])
PIVOT_RANKS = np.array([int(float(s)) for s in _PIVOT_ORDER])


def _row_sum(row: np.ndarray) -> float:
    """DataFrame.sum(axis=1) over the pivot row in column order, NaN -> 0 (nansum)."""
    return np_sum(np.where(np.isnan(row), 0.0, row))


def top_stocks(date, vals):
    """KKT:356-373: factor-weighted top-10 by descending rank, per return type + cumsum."""
    off = group_starts(date)
    nd = len(off) - 1
    res = np.zeros((nd, len(RETURN_TYPES)))
    for g in range(nd):
        s, e = off[g], off[g + 1]
        rk = rank_first(vals[s:e, 0], ascending=False)
        piv = np.full((len(RETURN_TYPES) + 1, TOP_K), np.nan)
        for c, r in enumerate(PIVOT_RANKS):
            hit = np.flatnonzero(rk == r)
            if len(hit):
                piv[:, c] = vals[s + hit[0], :]
        w = piv[0] / _row_sum(piv[0])
        for k in range(len(RETURN_TYPES)):
            res[g, k] = _row_sum(piv[1 + k] * w)
    cum = np.cumsum(res, axis=0)
    dates = date[off[:-1]]
    od, ot, ov = [], [], []
    names = list(RETURN_TYPES) + [f"cum_{r}" for r in RETURN_TYPES]
    full = np.concatenate([res, cum], axis=1)
    for i in range(nd):
        for j, nm in enumerate(names):
            od.append(dates[i]); ot.append(nm); ov.append(full[i, j])
    return np.array(od), np.array(ot), np.array(ov, dtype=np.float64)


def analyze(sig_date, sig_id, sig_val, px_date, px_id, px_close) -> dict:
    """AlphaSignalAnalyzer.run() minus plotting (KKT:298-305)."""
    d, i, v = add_returns(sig_date, sig_id, sig_val, px_date, px_id, px_close)
    out = {"fr_date": d, "fr_id": i, "fr_vals": v}
    out["ic_date"], out["ic_type"], out["ic"] = ic_series(d, v)
    out["ir_year"], out["ir_type"], out["ir"] = ir_table(out["ic_date"], out["ic_type"], out["ic"])
    for k, rt in enumerate(RETURN_TYPES):
        (ld, ll, lv), (sd, sl, sv) = layers(d, v, 1 + k)
        out[f"lay_{rt}_date"], out[f"lay_{rt}_layer"], out[f"lay_{rt}"] = ld, ll, lv
        out[f"ls_{rt}_date"], out[f"ls_{rt}_layer"], out[f"ls_{rt}"] = sd, sl, sv
    out["pt_date"], out["pt_type"], out["pt_ret"] = top_stocks(d, v)
    return out

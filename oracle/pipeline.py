"""ORACLE -- test infrastructure only (see oracle/__init__.py).

Restatement of the notebook cells between the factor build and the models:

* split by date (``KKT:424-428``): train = date <= 2015-12-31, valid = [2015-12-31, 2016-12-31],
  test = date >= 2016-12-31 (``.loc`` slices are inclusive at both ends);
* feature columns = every column except the raw inputs and ``target``, in sorted name order
  (``Index.difference``, ``KKT:433-443``) -- this includes ``tmr_ret1d``, as the reference does;
* per-security z-score with train-window mean (pandas group_mean, Kahan) and std (group_var,
  Welford, ddof=1), inf -> NaN, dropna (``KKT:449-458``);
* pooled OLS (``KKT:582-590``): scikit-learn ``LinearRegression`` -- the reference's own
  dependency, present in this image -- is the oracle for R1.
Pinned against tests/golden/zscore_pipeline.npz and ols_pipeline.npz.
"""
from __future__ import annotations

import numpy as np

from . import _p, lib

EXCLUDED = ("close_price", "excess_ret1d", "group_id", "in_trading_universe", "ret1d", "volume",
            "target")


def feature_columns(columns) -> list:
    return sorted(c for c in columns if c not in EXCLUDED)


def split_masks(date_ns: np.ndarray, train_end="2015-12-31", valid_end="2016-12-31"):
    d = np.asarray(date_ns).astype("datetime64[ns]")
    te, ve = np.datetime64(train_end, "ns"), np.datetime64(valid_end, "ns")
    return d <= te, (d >= te) & (d <= ve), d >= ve


def group_stats(ids: np.ndarray, X: np.ndarray, uid: np.ndarray):
    """groupby('security_id').mean() / .std() over rows (ids, X) -> [len(uid)][K] each."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    n, K = X.shape
    lab = np.searchsorted(uid, ids).astype(np.int64)
    lab[(lab >= len(uid)) | (uid[np.minimum(lab, len(uid) - 1)] != ids)] = -1
    G = len(uid)
    a, b = np.zeros(G * K), np.zeros(G * K)
    nobs = np.zeros(G * K, dtype=np.int64)
    mu, sd = np.zeros(G * K), np.zeros(G * K)
    L = lib()
    L.oracle_group_mean2(n, K, _p(lab), _p(X), G, _p(a), _p(b), _p(nobs), _p(mu))
    L.oracle_group_std(n, K, _p(lab), _p(X), G, _p(a), _p(nobs), _p(sd))
    return mu.reshape(G, K), sd.reshape(G, K)


def zscore(ids: np.ndarray, X: np.ndarray, uid: np.ndarray, mu: np.ndarray, sd: np.ndarray):
    """(x - mu[id]) / sigma[id], inf -> NaN; returns (z, keep) with keep = no NaN in the row."""
    j = np.searchsorted(uid, ids)
    ok = (j < len(uid))
    j = np.minimum(j, len(uid) - 1)
    ok &= uid[j] == ids
    with np.errstate(all="ignore"):
        z = (X - mu[j]) / sd[j]
    z[~ok] = np.nan
    z[np.isinf(z)] = np.nan
    return z, ~np.isnan(z).any(axis=1)


def pooled_ols(X: np.ndarray, y: np.ndarray):
    """sklearn LinearRegression().fit(X, y) -> (intercept, coef)."""
    from sklearn.linear_model import LinearRegression
    m = LinearRegression().fit(X, y)
    return float(np.ravel(m.intercept_)[0]), np.ravel(m.coef_).astype(np.float64)


def xs_ols(date: np.ndarray, X: np.ndarray, y: np.ndarray):
    """Per-date OLS with intercept (the north-star Fama-MacBeth extension; the reference has no
    per-date regression -- SURVEY.md §0 F5 -- so this oracle is numpy lstsq, parity unpinned by
    the reference).  Returns (dates, beta[T][p+1], n[T])."""
    order = np.argsort(date, kind="stable")
    date, X, y = date[order], X[order], y[order]
    cut = np.flatnonzero(np.r_[True, date[1:] != date[:-1]])
    off = np.r_[cut, len(date)]
    B, N = [], []
    for g in range(len(off) - 1):
        s, e = off[g], off[g + 1]
        A = np.column_stack([np.ones(e - s), X[s:e]])
        # equilibrated columns (raw factors span ~1e9 in scale: an unscaled lstsq loses the
        # small columns' digits), solved, then unscaled
        sc = np.sqrt((A * A).sum(axis=0))
        sc[sc == 0] = 1.0
        beta, *_ = np.linalg.lstsq(A / sc, y[s:e], rcond=None)
        B.append(beta / sc)
        N.append(e - s)
    return date[off[:-1]], np.array(B), np.array(N)


def fama_macbeth(beta: np.ndarray):
    """mean_t beta_t and t = mean / (std / sqrt(T)) (ddof 1)."""
    T = beta.shape[0]
    m = beta.mean(axis=0)
    s = beta.std(axis=0, ddof=1)
    return m, m / (s / np.sqrt(T))

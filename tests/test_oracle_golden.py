"""The oracle against the reference's own outputs (tests/golden/*.npz, made by make_golden.py).

Bit-exact everywhere the reference is deterministic; the pooled OLS on the notebook's
rank-deficient 97-column design is compared at 1e-6 (sklearn's threaded LAPACK is not
reproducible to the bit there); the weight solve is the exact QP (see oracle/portfolio.py).
"""
import os

import numpy as np
import pandas as pd
import pytest

import oracle
from oracle import pipeline as PL
from oracle import portfolio as P
from oracle import xs


def same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape:
        return False
    if a.dtype.kind == "f":
        return bool(((a == b) | (np.isnan(a) & np.isnan(b))).all())
    return bool((a == b).all())


def frame_from(g):
    return pd.DataFrame({
        "data_date": g["in_date"].astype("datetime64[ns]"), "security_id": g["in_id"],
        "close_price": g["in_close"], "volume": g["in_volume"], "ret1d": g["in_ret1d"],
        "excess_ret1d": g["in_excess"], "group_id": g["in_group"],
        "in_trading_universe": np.where(g["in_tradable"], "Y", "N")})


@pytest.mark.parametrize("name", ["edge", "scales", "pipeline"])
def test_factors_bit_exact(golden_dir, name):
    g = np.load(os.path.join(golden_dir, f"factors_{name}.npz"))
    out = oracle.compute_factors(frame_from(g))
    assert list(g["all_cols"]) == oracle.FACTOR_NAMES
    assert np.array_equal(out.index.values, g["out_index"])          # pre-dropna RangeIndex
    assert np.array_equal(out["security_id"].values, g["out_id"])
    cols = list(g["out_cols"])
    assert same(out[cols].to_numpy(np.float64), g["out"])


@pytest.mark.parametrize("name", ["zfactor", "lrpred"])
def test_analyzer_bit_exact(golden_dir, name):
    g = np.load(os.path.join(golden_dir, f"analyzer_{name}.npz"))
    o = xs.analyze(g["sig_date"], g["sig_id"], g["sig_val"], g["px_date"], g["px_id"], g["px_close"])
    keys = ["fr_date", "fr_id", "fr_vals", "ic_date", "ic_type", "ic", "ir_year", "ir_type", "ir",
            "pt_date", "pt_type", "pt_ret"]
    for rt in xs.RETURN_TYPES:
        keys += [f"lay_{rt}_date", f"lay_{rt}_layer", f"lay_{rt}", f"ls_{rt}_date",
                 f"ls_{rt}_layer", f"ls_{rt}"]
    for k in keys:
        assert same(o[k], g[k]), k


def test_portfolio_bit_exact(golden_dir):
    g = np.load(os.path.join(golden_dir, "portfolio_pipeline.npz"))
    o = P.run_portfolio(g["pred_date"], g["pred_id"], g["pred"], g["hist_date"], g["hist_id"],
                        g["hist"], g["all_date"], g["all_id"], g["all_tradable"], g["all_close"],
                        g["all_tmr"])
    for k in ("value", "turnover", "long_ret", "short_ret"):
        assert same(o[k], g[k]), k
    assert same(np.concatenate(o["books"]), g["book_ids"])
    assert same(np.concatenate(o["weights"]), g["book_w"])
    assert P.sharpe(o["value"]) == g["sharpe"]
    assert P.annualized_return(o["value"]) == g["ann_ret"]
    assert P.max_drawdown(o["value"]) == g["mdd"]


@pytest.mark.parametrize("n", [10, 9, 20, 30])
def test_weights_vs_slsqp(golden_dir, n):
    g = np.load(os.path.join(golden_dir, "weights_cases.npz"))
    S = P.pairwise_cov(g[f"n{n}_ret"])
    assert same(S, g[f"n{n}_cov"])
    w, _ = P.box_qp_weights(S)
    sl = g[f"n{n}_slsqp"]
    if n == 10:
        assert same(w, sl)                           # unique feasible point: 0.1 exactly
    elif n == 9:
        assert same(w, np.full(9, 0.1))              # infeasible: SLSQP stops at the bound
        assert np.abs(w - sl).max() < 1e-9
    else:
        assert abs(w.sum() - 1) < 1e-14 and w.min() >= 0 and w.max() <= 0.1
        assert w @ S @ w <= sl @ S @ sl * (1 + 1e-12)   # exact optimum <= SLSQP's objective
        # KKT conditions of the exact optimum
        gr = S @ w
        free = (w > 1e-12) & (w < 0.1 - 1e-12)
        lam = -gr[free].mean()
        assert np.abs(gr[free] + lam).max() < 1e-12 * np.abs(gr).max()


def test_zscore_and_ols(golden_dir):
    g = np.load(os.path.join(golden_dir, "factors_pipeline.npz"))
    out = oracle.compute_factors(frame_from(g)).sort_values(["data_date", "security_id"])
    cols = PL.feature_columns(out.columns.drop(["data_date", "security_id"]))
    z = np.load(os.path.join(golden_dir, "zscore_pipeline.npz"))
    assert cols == list(z["x_cols"])
    d = out["data_date"].values.astype("datetime64[ns]").astype(np.int64)
    ids = out["security_id"].values
    X = out[cols].to_numpy(np.float64)
    y = out["target"].to_numpy()
    uid = np.unique(ids)
    tr, va, te = PL.split_masks(d)
    mu, sd = PL.group_stats(ids[tr], X[tr], uid)
    zc = [cols.index(c) for c in z["z_cols"]]
    parts = {}
    for nm, m in (("df_train_x", tr), ("df_valid_x", va), ("df_test_x", te)):
        zz, keep = PL.zscore(ids[m], X[m], uid, mu, sd)
        assert same(ids[m][keep], z[f"{nm}_id"]) and same(d[m][keep], z[f"{nm}_date"])
        assert same(zz[keep][:, zc], z[f"{nm}_vals"])
        parts[nm] = (zz[keep], y[m][keep])
    o = np.load(os.path.join(golden_dir, "ols_pipeline.npz"))
    Xtr = np.vstack([parts["df_train_x"][0], parts["df_valid_x"][0]])
    ytr = np.r_[parts["df_train_x"][1], parts["df_valid_x"][1]]
    sub = [cols.index(c) for c in o["sub_cols"]]
    a1, c1 = PL.pooled_ols(Xtr[:, sub], ytr)
    assert a1 == o["sub_intercept"][0] and same(c1, o["sub_coef"])
    a0, c0 = PL.pooled_ols(Xtr, ytr)
    assert abs(a0 - o["full_intercept"][0]) < 1e-6 and np.abs(c0 - o["full_coef"]).max() < 1e-6


def test_np_sum_matches_numpy_buffered_reduce():
    """oracle np_sum = numpy's own np.add.reduce (pandas Series.sum / mean, KKT:315-318, the
    turnover sum of KKT:887) -- including vectors longer than numpy's 8192-element reduction
    buffer, where the result is NOT one pairwise tree (the per-date groups and id unions of the
    10,000-asset config are ~9,000-10,000 long)."""
    from oracle.xs import np_sum
    # The chunking is numpy's ufunc buffer size (np.getbufsize(), NPY_BUFSIZE), an implementation
    # detail the reference does not pin: verified against numpy 2.2.6 (the goldens' version,
    # DESIGN.md §2).  Another numpy with another buffer size fails HERE, by name, instead of the
    # engine silently diverging from it on vectors over 8192 elements.
    assert np.getbufsize() == 8192, (
        f"numpy {np.__version__}: ufunc buffer size {np.getbufsize()} != 8192 -- the engine and "
        f"oracle model numpy 2.2.6's 8192-element buffered reduction (oracle/xs_oracle.c)")
    rng = np.random.default_rng(12)
    for n in [0, 1, 7, 8, 127, 128, 129, 1000, 8191, 8192, 8193, 9000, 16384, 16385, 24577,
              40000]:
        for scale in (1.0, 1e-3, 1e8):
            v = rng.standard_normal(n) * scale * 10.0 ** rng.integers(-2, 3, n)
            assert np_sum(v) == np.sum(v), (f"numpy {np.__version__}: buffered reduce differs "
                                            f"from the 8192-chunk model", n, scale)
            sparse = np.where(rng.random(n) < 0.004, np.abs(v), 0.0)   # a turnover vector
            assert np_sum(sparse) == np.sum(sparse), (n, scale)

"""GPU parity of the rebalance / weights / PnL path (K1-K4) against the reference's own outputs
(bit-exact where the reference is deterministic) and the exact-QP oracle (rel 1e-9)."""
import os

import numpy as np
import pandas as pd
import pytest

from helpers import same

pytestmark = pytest.mark.gpu


def frames(g):
    pred = pd.DataFrame({"lr_predict": g["pred"]}, index=pd.MultiIndex.from_arrays(
        [g["pred_date"].astype("datetime64[ns]"), g["pred_id"]]))
    hist = pd.DataFrame({"target": g["hist"]}, index=pd.MultiIndex.from_arrays(
        [g["hist_date"].astype("datetime64[ns]"), g["hist_id"]]))
    all_df = pd.DataFrame({"in_trading_universe": np.where(g["all_tradable"], "Y", "N"),
                           "close_price": g["all_close"], "tmr_ret1d": g["all_tmr"]},
                          index=pd.MultiIndex.from_arrays(
                              [g["all_date"].astype("datetime64[ns]"), g["all_id"]],
                              names=["data_date", "security_id"]))
    return pred, hist, all_df


def test_portfolio_manager_matches_reference(golden_dir):
    from afm.portfolio import PortfolioManager
    g = np.load(os.path.join(golden_dir, "portfolio_pipeline.npz"))
    pred, hist, all_df = frames(g)
    pm = PortfolioManager(pred, hist, all_df)
    pm.calculate_portfolio()
    assert same(np.asarray(pm.portfolio_value["Portfolio"], dtype=np.float64), g["value"])
    assert same(np.asarray(pm.turnovers, dtype=np.float64), g["turnover"])
    assert same(np.asarray(pm.long_returns), g["long_ret"])
    assert same(np.asarray(pm.short_returns), g["short_ret"])
    ids = np.concatenate([np.r_[L, S] for _, L, S in pm.books]).astype(np.int64)
    assert same(ids, g["book_ids"])
    assert pm.calculate_sharpe_ratio() == g["sharpe"]
    assert pm.annualized_return() == g["ann_ret"]
    assert pm.max_drawdown() == g["mdd"]


@pytest.mark.parametrize("n", [10, 9, 20, 30])
def test_determine_weights(golden_dir, n):
    from afm.portfolio import min_variance_weights
    from oracle import portfolio as P
    g = np.load(os.path.join(golden_dir, "weights_cases.npz"))
    R = g[f"n{n}_ret"]
    w, cov = min_variance_weights(R)
    ref_cov = g[f"n{n}_cov"]
    if np.isnan(R).any():
        assert same(cov, ref_cov)                    # nancorr(cov=True): bit-exact Welford
    else:
        assert np.abs(cov - ref_cov).max() <= 1e-13 * np.abs(ref_cov).max()
    wo, _ = P.box_qp_weights(P.pairwise_cov(R))
    if n in (9, 10):
        assert same(w, np.full(n, 0.1))
    else:
        assert np.abs(w - wo).max() < 1e-9
        assert abs(w.sum() - 1) < 1e-13


@pytest.mark.parametrize("top_n,window", [(10, 60), (20, 120), (3, None)])
def test_rolling_window_books_vs_oracle(top_n, window):
    """North-star rolling history window and bounded (top_n > 10) books vs the oracle."""
    from afm.portfolio import PortfolioManager
    from oracle import portfolio as P
    rng = np.random.default_rng(top_n)
    T, A = 160, 48
    dates = np.asarray(np.busday_offset(np.datetime64("2016-01-04"), np.arange(T), roll="forward"),
                       dtype="datetime64[ns]")
    ids = 2000 + 3 * np.arange(A)
    present = rng.random((T, A)) < 0.93
    tt, aa = np.nonzero(present)
    d, i = dates[tt], ids[aa]
    ret = rng.normal(0, 0.02, len(tt))
    close = 50 * np.exp(rng.normal(0, 0.1, len(tt)))
    trad = rng.random(len(tt)) < 0.9
    hist_m = tt < 100
    test_m = tt >= 100
    pred_v = rng.normal(size=test_m.sum())
    pred = pd.DataFrame({"p": pred_v}, index=pd.MultiIndex.from_arrays([d[test_m], i[test_m]]))
    hist = pd.DataFrame({"target": ret[hist_m]}, index=pd.MultiIndex.from_arrays([d[hist_m], i[hist_m]]))
    all_df = pd.DataFrame({"in_trading_universe": np.where(trad, "Y", "N"), "close_price": close,
                           "tmr_ret1d": ret}, index=pd.MultiIndex.from_arrays([d, i]))
    pm = PortfolioManager(pred, hist, all_df, top_n=top_n, window=window)
    pm.calculate_portfolio()
    o = P.run_portfolio(d[test_m].astype(np.int64), i[test_m], pred_v,
                        d[hist_m].astype(np.int64), i[hist_m], ret[hist_m],
                        d.astype(np.int64), i, trad, close, ret, top_n=top_n,
                        window=window if window else None)
    # the oracle's rolling window counts history DATES; the GPU counts grid dates (the same here:
    # every calendar date carries history rows)
    for (dt, L, S), Lo, So in zip(pm.books, o["books"][0::2], o["books"][1::2]):
        assert L == Lo.tolist() and S == So.tolist()
    v = np.asarray(pm.portfolio_value["Portfolio"], dtype=np.float64)
    assert np.abs(v - o["value"]).max() / o["value"].max() < 1e-12
    assert np.abs(np.asarray(pm.turnovers, dtype=np.float64) - o["turnover"]).max() <= \
        1e-9 * max(1.0, o["turnover"].max())


@pytest.mark.parametrize("A,levels", [(48, 4), (300, 3), (12500, 7)])
def test_tied_predictions_books_vs_oracle(A, levels):
    """Predictions on a few discrete levels: the top/bottom-k threshold falls inside a tie, which
    the engine breaks by ascending asset index, like the oracle.  A = 12500 exceeds the register
    key capacity (12288) and takes the global-memory selection path."""
    from afm.portfolio import PortfolioManager
    from oracle import portfolio as P
    rng = np.random.default_rng(A)
    T = 130
    top_n = 10
    dates = np.asarray(np.busday_offset(np.datetime64("2016-01-04"), np.arange(T), roll="forward"),
                       dtype="datetime64[ns]")
    ids = 7 + 2 * np.arange(A)
    present = rng.random((T, A)) < 0.95
    tt, aa = np.nonzero(present)
    d, i = dates[tt], ids[aa]
    ret = rng.normal(0, 0.02, len(tt))
    close = 50 * np.exp(rng.normal(0, 0.1, len(tt)))
    trad = rng.random(len(tt)) < 0.9
    hist_m = tt < 100
    test_m = tt >= 100
    pred_v = rng.integers(0, levels, test_m.sum()) * 0.25 - 0.5
    pred = pd.DataFrame({"p": pred_v}, index=pd.MultiIndex.from_arrays([d[test_m], i[test_m]]))
    hist = pd.DataFrame({"target": ret[hist_m]}, index=pd.MultiIndex.from_arrays([d[hist_m], i[hist_m]]))
    all_df = pd.DataFrame({"in_trading_universe": np.where(trad, "Y", "N"), "close_price": close,
                           "tmr_ret1d": ret}, index=pd.MultiIndex.from_arrays([d, i]))
    pm = PortfolioManager(pred, hist, all_df, top_n=top_n, window=60)
    pm.calculate_portfolio()
    o = P.run_portfolio(d[test_m].astype(np.int64), i[test_m], pred_v,
                        d[hist_m].astype(np.int64), i[hist_m], ret[hist_m],
                        d.astype(np.int64), i, trad, close, ret, top_n=top_n, window=60)
    for (dt, L, S), Lo, So in zip(pm.books, o["books"][0::2], o["books"][1::2]):
        assert L == Lo.tolist() and S == So.tolist()


@pytest.mark.parametrize("top_n,window,npaths", [(10, 60, 37), (20, None, 8)])
def test_bootstrap_paths_vs_oracle(top_n, window, npaths):
    """Config E: bootstrap resamples of the rebalance dates (with replacement, repeated
    consecutive dates included); every path's value / turnover recursion vs the oracle's
    KKT:864-892 restatement over the same date sequence.  The identity path reproduces
    calculate_portfolio.  top_n = 10 (weights exactly 0.1): bit-exact; top_n = 20 (active-set
    QP weights, rel 1e-9 vs the oracle): the values at rel 1e-12."""
    from afm.portfolio import PortfolioManager
    from oracle import portfolio as P
    rng = np.random.default_rng(100 + top_n)
    T, A = 150, 70
    dates = np.asarray(np.busday_offset(np.datetime64("2016-01-04"), np.arange(T), roll="forward"),
                       dtype="datetime64[ns]")
    ids = 300 + 5 * np.arange(A)
    present = rng.random((T, A)) < 0.9
    present[140, :] = False
    present[140, :30] = True                                      # a thin date: k = n // 2
    tt, aa = np.nonzero(present)
    d, i = dates[tt], ids[aa]
    ret = rng.normal(0, 0.02, len(tt))
    close = 50 * np.exp(rng.normal(0, 0.1, len(tt)))
    trad = rng.random(len(tt)) < 0.9
    hist_m = tt < 100
    test_m = tt >= 100
    pred_v = rng.normal(size=test_m.sum())
    pred = pd.DataFrame({"p": pred_v}, index=pd.MultiIndex.from_arrays([d[test_m], i[test_m]]))
    hist = pd.DataFrame({"target": ret[hist_m]}, index=pd.MultiIndex.from_arrays([d[hist_m], i[hist_m]]))
    all_df = pd.DataFrame({"in_trading_universe": np.where(trad, "Y", "N"), "close_price": close,
                           "tmr_ret1d": ret}, index=pd.MultiIndex.from_arrays([d, i]))
    pm = PortfolioManager(pred, hist, all_df, top_n=top_n, window=window)
    nd = 50
    paths = np.random.default_rng(2023).integers(0, nd, size=(npaths, nd)).astype(np.int32)
    paths[1, 5:9] = 17                                            # repeated consecutive dates
    paths[2] = np.arange(nd)                                      # the plain sequence
    got_paths, got = pm.bootstrap(paths=paths)
    assert (got_paths == paths).all()
    o = P.run_bootstrap(paths, d[test_m].astype(np.int64), i[test_m], pred_v,
                        d[hist_m].astype(np.int64), i[hist_m], ret[hist_m], d.astype(np.int64), i,
                        trad, close, ret, top_n=top_n, window=window)
    if top_n == 10:
        for k in ("value", "turnover", "long_ret", "short_ret"):
            assert same(got[k], o[k]), k
    else:
        assert np.abs(got["value"] - o["value"]).max() / o["value"].max() < 1e-12
        assert np.abs(got["turnover"] - o["turnover"]).max() <= 1e-9 * max(1.0, o["turnover"].max())
    pm.calculate_portfolio()
    v = np.asarray(pm.portfolio_value["Portfolio"], dtype=np.float64)
    assert same(got["value"][2], v)
    assert same(got["turnover"][2, 1:], np.asarray(pm.turnovers[1:], dtype=np.float64))


@pytest.mark.parametrize("k,holes", [(33, False), (37, True), (50, False), (64, False),
                                     (100, False), (100, True), (127, True), (128, False)])
def test_large_book_weights_vs_oracle(k, holes):
    """determine_weights for the survey's stress book sizes (top_n = 100): the
    workgroup active-set QP (S_FF^-1 in registers, four-pivot block sweep -- sizes that are not
    a multiple of 4 pad the last block) and the one-pass MFMA covariance against the oracle's
    refactor-every-step solve, rel 1e-9; identical bound sets."""
    from afm.portfolio import min_variance_weights
    from oracle import portfolio as P
    rng = np.random.default_rng(k + holes)
    rows = 260
    f = rng.normal(0, 0.01, (rows, 4))                       # a few common factors + noise
    scale = rng.uniform(0.3, 2, k)
    scale[:3] = 0.05                                         # low-vol names: pinned at hi
    R = f @ rng.normal(0, 0.2, (4, k)) + rng.normal(0, 0.02, (rows, k)) * scale
    if holes:
        R[rng.random(R.shape) < 0.01] = np.nan
    w, cov = min_variance_weights(R)
    S = P.pairwise_cov(R)
    assert np.abs(cov - S).max() <= 1e-12 * np.abs(S).max()
    wo, it = P.box_qp_weights(S)
    assert it >= 3                                           # the active set really iterates
    assert (wo >= 0.1 - 1e-14).any() and (wo <= 1e-14).any()    # both bounds active
    assert np.array_equal(w <= 1e-14, wo <= 1e-14)
    assert np.array_equal(w >= 0.1 - 1e-14, wo >= 0.1 - 1e-14)
    assert np.abs(w - wo).max() < 1e-9
    assert abs(w.sum() - 1) < 1e-12


def test_top100_books_weights_pnl_vs_oracle():
    """Rebalance at top_n = 100 (the stress book, KKT:796 parameterised): books identical, weights
    rel 1e-9 against the exact-QP oracle, the value path rel 1e-12."""
    from afm.portfolio import PortfolioManager
    from oracle import portfolio as P
    rng = np.random.default_rng(100)
    T, A, top_n = 190, 420, 100
    dates = np.asarray(np.busday_offset(np.datetime64("2016-01-04"), np.arange(T), roll="forward"),
                       dtype="datetime64[ns]")
    ids = 11 + 3 * np.arange(A)
    present = rng.random((T, A)) < 0.97
    present[:170] = True                                     # complete history: np.cov path
    tt, aa = np.nonzero(present)
    d, i = dates[tt], ids[aa]
    f = rng.normal(0, 0.01, (T, 3))
    ret = (f @ rng.normal(0, 1, (3, A)))[tt, aa] + rng.normal(0, 0.02, len(tt))
    close = 50 * np.exp(rng.normal(0, 0.1, len(tt)))
    trad = rng.random(len(tt)) < 0.95
    hist_m = tt < 170
    test_m = tt >= 170
    pred_v = rng.normal(size=test_m.sum())
    pred = pd.DataFrame({"p": pred_v}, index=pd.MultiIndex.from_arrays([d[test_m], i[test_m]]))
    hist = pd.DataFrame({"target": ret[hist_m]}, index=pd.MultiIndex.from_arrays([d[hist_m], i[hist_m]]))
    all_df = pd.DataFrame({"in_trading_universe": np.where(trad, "Y", "N"), "close_price": close,
                           "tmr_ret1d": ret}, index=pd.MultiIndex.from_arrays([d, i]))
    pm = PortfolioManager(pred, hist, all_df, top_n=top_n, window=120)
    pm.calculate_portfolio()
    o = P.run_portfolio(d[test_m].astype(np.int64), i[test_m], pred_v,
                        d[hist_m].astype(np.int64), i[hist_m], ret[hist_m],
                        d.astype(np.int64), i, trad, close, ret, top_n=top_n, window=120)
    for (dt, L, S), Lo, So in zip(pm.books, o["books"][0::2], o["books"][1::2]):
        assert len(L) == top_n
        assert L == Lo.tolist() and S == So.tolist()
    for j, (wol, wos) in enumerate(zip(o["weights"][0::2], o["weights"][1::2])):
        assert np.abs(pm.weights[j, 0, :top_n] - wol).max() < 1e-9
        assert np.abs(pm.weights[j, 1, :top_n] - wos).max() < 1e-9
    v = np.asarray(pm.portfolio_value["Portfolio"], dtype=np.float64)
    assert np.abs(v - o["value"]).max() / o["value"].max() < 1e-12


@pytest.mark.parametrize("A", [9800])
def test_large_union_turnover_vs_numpy_reduce(A):
    """Prediction-id unions of ~9,800 names (config C scale): numpy's np.add.reduce sums over its
    8192-element buffers one by one, so the turnover sum (Series.sum, KKT:887) is not one pairwise
    tree.  The engine's turnover DAG (np_lca_depth) and the oracle (np_sum, pinned to numpy) must
    agree bit for bit on turnover and value."""
    from afm.portfolio import PortfolioManager
    from oracle import portfolio as P
    rng = np.random.default_rng(A)
    T, top_n = 112, 10
    dates = np.asarray(np.busday_offset(np.datetime64("2016-01-04"), np.arange(T), roll="forward"),
                       dtype="datetime64[ns]")
    ids = 5 + 2 * np.arange(A)
    present = rng.random((T, A)) < 0.97
    tt, aa = np.nonzero(present)
    d, i = dates[tt], ids[aa]
    ret = rng.normal(0, 0.02, len(tt))
    close = 50 * np.exp(rng.normal(0, 0.1, len(tt)))
    trad = rng.random(len(tt)) < 0.9
    hist_m = tt < 100
    test_m = tt >= 100
    pred_v = rng.normal(size=test_m.sum())
    pred = pd.DataFrame({"p": pred_v}, index=pd.MultiIndex.from_arrays([d[test_m], i[test_m]]))
    hist = pd.DataFrame({"target": ret[hist_m]}, index=pd.MultiIndex.from_arrays([d[hist_m], i[hist_m]]))
    all_df = pd.DataFrame({"in_trading_universe": np.where(trad, "Y", "N"), "close_price": close,
                           "tmr_ret1d": ret}, index=pd.MultiIndex.from_arrays([d, i]))
    pm = PortfolioManager(pred, hist, all_df, top_n=top_n, window=60)
    pm.calculate_portfolio()
    o = P.run_portfolio(d[test_m].astype(np.int64), i[test_m], pred_v,
                        d[hist_m].astype(np.int64), i[hist_m], ret[hist_m],
                        d.astype(np.int64), i, trad, close, ret, top_n=top_n, window=60)
    for (dt, L, S), Lo, So in zip(pm.books, o["books"][0::2], o["books"][1::2]):
        assert L == Lo.tolist() and S == So.tolist()
    assert same(np.asarray(pm.turnovers, dtype=np.float64), o["turnover"])
    assert same(np.asarray(pm.portfolio_value["Portfolio"], dtype=np.float64), o["value"])


def test_large_book_full_history_window_vs_oracle():
    """Books over 32 names with no rolling window (the reference's whole training history,
    KKT:858-859) whose history starts after the first grid date: the member-major history panel
    is staged from that later start."""
    from afm.portfolio import PortfolioManager
    from oracle import portfolio as P
    rng = np.random.default_rng(41)
    T, A, top_n = 150, 160, 40
    dates = np.asarray(np.busday_offset(np.datetime64("2016-01-04"), np.arange(T), roll="forward"),
                       dtype="datetime64[ns]")
    ids = 3 + 7 * np.arange(A)
    present = rng.random((T, A)) < 0.96
    tt, aa = np.nonzero(present)
    d, i = dates[tt], ids[aa]
    f = rng.normal(0, 0.01, (T, 3))
    ret = (f @ rng.normal(0, 1, (3, A)))[tt, aa] + rng.normal(0, 0.02, len(tt))
    close = 50 * np.exp(rng.normal(0, 0.1, len(tt)))
    trad = rng.random(len(tt)) < 0.95
    hist_m = (tt >= 23) & (tt < 130)                    # history from grid date 23 on
    test_m = tt >= 130
    pred_v = rng.normal(size=test_m.sum())
    pred = pd.DataFrame({"p": pred_v}, index=pd.MultiIndex.from_arrays([d[test_m], i[test_m]]))
    hist = pd.DataFrame({"target": ret[hist_m]}, index=pd.MultiIndex.from_arrays([d[hist_m], i[hist_m]]))
    all_df = pd.DataFrame({"in_trading_universe": np.where(trad, "Y", "N"), "close_price": close,
                           "tmr_ret1d": ret}, index=pd.MultiIndex.from_arrays([d, i]))
    pm = PortfolioManager(pred, hist, all_df, top_n=top_n, window=None)
    pm.calculate_portfolio()
    o = P.run_portfolio(d[test_m].astype(np.int64), i[test_m], pred_v,
                        d[hist_m].astype(np.int64), i[hist_m], ret[hist_m],
                        d.astype(np.int64), i, trad, close, ret, top_n=top_n, window=None)
    for (dt, L, S), Lo, So in zip(pm.books, o["books"][0::2], o["books"][1::2]):
        assert L == Lo.tolist() and S == So.tolist()
    for j, (wol, wos) in enumerate(zip(o["weights"][0::2], o["weights"][1::2])):
        assert np.abs(pm.weights[j, 0, :top_n] - wol).max() < 1e-9
        assert np.abs(pm.weights[j, 1, :top_n] - wos).max() < 1e-9
    v = np.asarray(pm.portfolio_value["Portfolio"], dtype=np.float64)
    assert np.abs(v - o["value"]).max() / o["value"].max() < 1e-12

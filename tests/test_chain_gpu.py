"""The benchmarked chain (afm.pipeline.Pipeline.step) against the CPU oracle chain at BASELINE
config A (500 assets x 10 years, all 97 features, window 252, top_n 10):

* live oracle (factors, z-score, scikit-learn Lasso, predict): z-score row set identical, Lasso
  fit size / iterations / support identical, coefficients and predictions within rel 1e-12;
* golden vectors (tests/golden/chain_A.npz, oracle/chain.py): books bit-exact on every rebalance
  date, weights rel 1e-9, PnL value path rel 1e-12, analyzer IC / top-10 series rel 1e-12,
  per-date FM betas rel 1e-9 on well-determined dates.
"""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))


@pytest.fixture(scope="module")
def chain_a():
    import torch
    import afm
    from afm.pipeline import Pipeline, PipelineConfig
    from afm.synthetic import make_panel
    from make_chain_golden import CONFIG_A as C
    p = make_panel(C["assets"], C["days"], seed=C["seed"], tradable_p=C["tradable_p"])
    grid = afm.PanelGrid.from_panel(p)
    pipe = Pipeline(grid, PipelineConfig(train_end=C["train_end"], valid_end=C["valid_end"],
                                         window=C["window"], top_n=C["top_n"]))
    pipe.step()
    torch.cuda.synchronize()
    gold = np.load(os.path.join(HERE, "golden", "chain_A.npz"))
    return p, pipe, gold, C


def test_lasso_and_predictions_vs_live_oracle(chain_a):
    from afm.grid import unpack_bits
    from oracle import chain
    p, pipe, gold, C = chain_a
    r = chain.run_chain(p, C["train_end"], C["valid_end"], portfolio=False, analyzer=False,
                        fm=False)
    # the z-score dropna row set (bit-exact)
    zr = unpack_bits(pipe.zrows, pipe.T).cpu().numpy()
    ref = np.zeros_like(zr)
    ref[r["zrows_t"], r["zrows_a"]] = True
    assert np.array_equal(zr, ref)
    # train-window statistics: pandas-exact kernels
    mu, sd = pipe.mu.cpu().numpy()[:, :p.A], pipe.sd.cpu().numpy()[:, :p.A]
    ok = np.isfinite(r["mu"].T)
    assert np.array_equal(mu[ok], r["mu"].T[ok])
    ok = np.isfinite(r["sd"].T)
    assert np.array_equal(sd[ok], r["sd"].T[ok])
    # Lasso: fit rows (train_end counted twice), iterations, support, coefficients
    s = pipe.summary()
    assert r["n_fit"] == int(gold["n_fit"])
    assert s["lasso_n_iter"] == r["n_iter"]
    b = s["lasso_beta"]
    assert np.array_equal(b[1:] != 0, r["coef"] != 0)
    assert np.abs(b[1:] - r["coef"]).max() <= 1e-12 * np.abs(r["coef"]).max()
    assert abs(b[0] - r["intercept"]) <= 1e-12 * max(abs(r["intercept"]), 1e-300) + 1e-18
    # predictions on exactly the test rows
    pred = pipe.pred.cpu().numpy()
    got = pred[r["pred_t"], r["pred_a"]]
    assert np.abs(got - r["pred"]).max() <= 1e-12 * np.abs(r["pred"]).max()
    mask = np.zeros_like(zr)
    mask[r["pred_t"], r["pred_a"]] = True
    assert np.isnan(pred[~mask]).all()


def test_books_weights_pnl_vs_golden(chain_a):
    p, pipe, gold, C = chain_a
    rd = pipe.rdates.cpu().numpy()
    dint = p.dates.astype("datetime64[ns]").astype(np.int64)
    assert np.array_equal(dint[rd], gold["reb_dates"])
    k = pipe.reb["k"].cpu().numpy()
    books = pipe.reb["books"].cpu().numpy()
    w = pipe.reb["weights"].cpu().numpy()
    gb, gw = gold["books"], gold["weights"]
    assert (k == C["top_n"]).all()
    assert (pipe.reb["status"].cpu().numpy() == 0).all()
    for i in range(len(rd)):
        for s in range(2):
            assert books[i, s, :k[i]].tolist() == gb[i, s, :k[i]].tolist(), (i, s)
    np.testing.assert_allclose(w[:, :, :C["top_n"]], gw, rtol=1e-9, atol=1e-12)
    v = pipe.pnl["value"].cpu().numpy()
    np.testing.assert_allclose(v, gold["value"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(pipe.pnl["turnover"].cpu().numpy(), gold["turnover"], rtol=1e-12,
                               atol=1e-6)
    np.testing.assert_allclose(pipe.pnl["long_ret"].cpu().numpy(), gold["long_ret"],
                               rtol=1e-12, atol=1e-15)


def test_analyzer_series_vs_golden(chain_a):
    p, pipe, gold, C = chain_a
    an = pipe.an
    ic = an["ic"].cpu().numpy()
    d = pipe.an_dates.cpu().numpy() + pipe.an_a0
    dint = p.dates.astype("datetime64[ns]").astype(np.int64)
    types = {"return_1": 0, "return_2": 1, "return_5": 2}
    pos = {x: i for i, x in enumerate(dint[d].tolist())}
    got = np.array([ic[pos[int(dt)], types[t]] for dt, t in zip(gold["ic_date"], gold["ic_type"])])
    np.testing.assert_allclose(got, gold["ic"], rtol=1e-12, atol=1e-14)
    # no IC where the oracle has none
    assert np.isfinite(ic).sum() == len(gold["ic"])
    # top-10 factor-weighted returns + their cumsum, on the dates with analyzer rows (the
    # reference's port_ret_df has no row for a date whose rows all drop, KKT:313-319)
    nr = an["nrows"].cpu().numpy()[pipe.an_dates.cpu().numpy()]
    live = nr > 0
    got = np.concatenate([an["port"].cpu().numpy(), an["cum_port"].cpu().numpy()],
                         axis=1)[live].reshape(-1)
    np.testing.assert_allclose(got, gold["pt_ret"], rtol=1e-10, atol=1e-13)


def test_fama_macbeth_vs_golden(chain_a):
    p, pipe, gold, C = chain_a
    fb = pipe.fm_beta.cpu().numpy()
    n = pipe.fm_nobs.cpu().numpy()
    rk = pipe.fm_rank.cpu().numpy()
    d, B, N = gold["fm_dates"], gold["fm_beta"], gold["fm_n"]
    assert np.array_equal(n[d].astype(np.int64), N)
    pf = len(pipe.cfg.fm_features)
    ok = N > 3 * pf                                   # well-determined dates
    assert ok.sum() > 0.8 * len(N)
    assert (rk[d[ok]] == pf).all()
    err = np.abs(fb[d[ok]] - B[ok]).max(axis=1) / np.abs(B[ok]).max(axis=1)
    assert err.max() < 1e-9, err.max()


@pytest.mark.parametrize("place", [{"labels_side": False}, {"fm_fork": "gram"},
                                   {"fm_fork": "rebalance"}, {"fm_free_cus": 8},
                                   {"early_zstats": True, "zstats_slabs": 0},
                                   {"early_zstats": True, "labels_side": False, "zstats_slabs": 0},
                                   {"early_fwd": False}, {"zstats_slabs": 0},
                                   {"zstats_slabs": 3}, {"zstats_slabs": 6, "labels_side": False}])
def test_stream_placement_bit_identical(chain_a, place):
    """The side-stream placements (label planes beside the factor kernel, the FM fork point) move
    work between streams only: the step's outputs are bitwise those of the default placement.
    early_zstats builds the panel in two time slabs with the z statistics between them;
    zstats_slabs streams the z statistics slab by slab behind the factor slabs (the default on
    this 500-asset grid: the reference step runs it, zstats_slabs = 0 is the one-pass path)."""
    import torch
    from afm.pipeline import Pipeline, PipelineConfig
    p, pipe, gold, C = chain_a
    other = Pipeline(pipe.g, PipelineConfig(train_end=C["train_end"], valid_end=C["valid_end"],
                                            window=C["window"], top_n=C["top_n"], **place))
    other.step()
    torch.cuda.synchronize()
    assert pipe.stream_z                              # the auto rule on a 500-asset grid
    if place.get("early_zstats"):
        assert other.early and 0 < other.ta < other.T
    if place.get("zstats_slabs", -1) >= 2:
        assert other.stream_z and len(other.zbounds) - 1 == place["zstats_slabs"]
    if place.get("zstats_slabs", -1) == 0:
        assert not other.stream_z
    for name in ("out", "pred", "lasso_beta", "fm_beta", "zs", "nanfree", "finite", "alldf",
                 "frows", "zrows", "pool_g"):
        a, b = getattr(pipe, name), getattr(other, name)
        assert torch.equal(a.view(torch.int64), b.view(torch.int64)), name
    for k in ("k", "books", "weights"):
        assert torch.equal(pipe.reb[k], other.reb[k]), k
    assert torch.equal(pipe.pnl["value"], other.pnl["value"])

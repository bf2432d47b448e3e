"""The end-to-end pipeline (bench step) against the oracle chain on a small panel: per-date betas
and the pooled OLS within rel 1e-9, books bit-exact given the engine's predictions, PnL path
within rel 1e-12."""
import numpy as np
import pytest

from helpers import oracle_panel

pytestmark = pytest.mark.gpu

WELL = ["RSI_14", "sd_5", "corr_15", "PSY", "ROCR_20", "volsd5_15", "MACD_12_24"]


def test_pipeline_vs_oracle_chain():
    import torch
    import afm
    from afm.pipeline import Pipeline, PipelineConfig
    from afm.synthetic import make_panel
    from oracle import pipeline as PL
    from oracle import portfolio as PF
    p = make_panel(150, 420, seed=21, tradable_p=0.9)
    grid = afm.PanelGrid.from_panel(p)
    cols = [afm.FACTOR_NAMES.index(c) for c in WELL]
    cfg = PipelineConfig(cols=cols, window=120, top_n=10)
    pipe = Pipeline(grid, cfg)
    pipe.step()
    torch.cuda.synchronize()

    tt, aa, fac = oracle_panel(p)
    X, y = fac[:, cols], fac[:, 96]
    fin = np.isfinite(fac[:, :96]).all(axis=1)
    use = fin & np.isfinite(y)
    # per-date betas
    d, B, N = PL.xs_ols(tt[use], X[use], y[use])
    beta = pipe.beta.cpu().numpy()
    ok = N > len(cols) + 5
    err = np.abs(beta[d[ok]] - B[ok]).max(axis=1) / np.abs(B[ok]).max(axis=1)
    assert err.max() < 1e-9, err.max()
    # pooled OLS over the train+valid dates
    tv = use & (tt < pipe.t_test)
    b0, b = PL.pooled_ols(X[tv], y[tv])
    pb = pipe.pool_beta[0].cpu().numpy()
    ref = np.r_[b0, b]
    assert np.abs(pb - ref).max() / np.abs(ref).max() < 1e-9
    # predictions on the test dates
    pred = pipe.pred.cpu().numpy()
    te = use & (tt >= pipe.t_test) & (tt < grid.T - 1)
    pv = pred[tt[te], aa[te]]
    pref = b0 + X[te] @ b
    assert np.abs(pv - pref).max() / np.abs(pref).max() < 1e-9
    other = np.ones_like(pred, dtype=bool)
    other[tt[te], aa[te]] = False
    assert np.isnan(pred[other]).all()
    # books + PnL from the engine's own predictions through the oracle portfolio
    ids = p.ids[aa]
    dates = p.dates[tt].astype(np.int64)
    o = PF.run_portfolio(dates[te], ids[te], pv, dates, ids, y, dates, ids,
                         p.tradable[tt, aa], p.close[tt, aa], fac[:, 97], window=120)
    k = pipe.reb["k"].cpu().numpy()
    books = pipe.reb["books"].cpu().numpy()
    for i in range(len(k)):
        assert p.ids[books[i, 0, :k[i]]].tolist() == o["books"][2 * i].tolist()
        assert p.ids[books[i, 1, :k[i]]].tolist() == o["books"][2 * i + 1].tolist()
    v = pipe.pnl["value"].cpu().numpy()
    assert np.abs(v - o["value"]).max() / o["value"].max() < 1e-12

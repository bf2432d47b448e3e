"""Full-size BASELINE configurations through the benchmarked chain (afm.pipeline.Pipeline), checked
against the oracle on sampled dates / paths (sizes where the whole oracle chain would take hours):

* C (10,000 assets x 5,040 days, 96 factors, window 252, top_n 10): every date's k, status and
  weights; the value path recomputed on the host by the oracle's KKT:864-892 recursion from the
  engine's books and PnL components (bit-exact); books vs oracle.portfolio.select_books on 24
  sampled dates from the engine's predictions; the pooled Gram vs torch fp64 D^T D, the Lasso
  vs the oracle's coordinate descent, predictions on 20 sampled dates.
* B (3,000 assets x 5,040 days, FM30): per-date Fama-MacBeth betas vs the oracle's lstsq on the
  same rows (rel 1e-9) and the IC series vs the oracle analyzer (oracle/xs.py) on sampled dates.
* E (1,024 bootstrap paths x 5,000 assets): sampled paths vs the oracle recursion over the same
  date sequence (bit-exact).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pipeline(assets, days, seed, **cfg):
    import torch
    import afm
    from afm.pipeline import Pipeline, PipelineConfig
    from afm.synthetic import make_panel
    p = make_panel(assets, days, seed=seed, tradable_p=0.9)
    grid = afm.PanelGrid.from_panel(p)
    pipe = Pipeline(grid, PipelineConfig(**cfg))
    pipe.step()
    torch.cuda.synchronize()
    return p, grid, pipe


def _records(pipe):
    """The oracle's per-date records (oracle/portfolio.py:_date_books fields) from the engine's
    books, prediction sets and PnL components."""
    pred = pipe.pred.cpu().numpy()
    rd = pipe.rdates.cpu().numpy()
    k = pipe.reb["k"].cpu().numpy()
    books = pipe.reb["books"].cpu().numpy()
    sums = pipe.reb["sums"].cpu().numpy()
    recs = []
    for i, t in enumerate(rd):
        ids = np.flatnonzero(~np.isnan(pred[t]))
        recs.append(dict(ids=ids, L=books[i, 0, :k[i]].astype(np.int64),
                         S=books[i, 1, :k[i]].astype(np.int64), lsum=sums[i, 0], ssum=sums[i, 1],
                         den_l=sums[i, 2], den_s=sums[i, 3]))
    return recs


@pytest.fixture(scope="module")
def config_c():
    return _pipeline(10000, 5040, 2023)


def test_config_c_books_weights_value(config_c):
    from afm.grid import unpack_bits
    from oracle import portfolio as P
    p, grid, pipe = config_c
    top_n = pipe.cfg.top_n
    k = pipe.reb["k"].cpu().numpy()
    st = pipe.reb["status"].cpu().numpy()
    w = pipe.reb["weights"].cpu().numpy()
    assert pipe.nd > 500 and (st == 0).all()
    assert (k == top_n).all()
    for s in range(2):
        ws = w[:, s, :top_n]
        assert ((ws >= 0) & (ws <= 0.1)).all()
        assert np.abs(ws.sum(axis=1) - 1).max() < 1e-12
    recs = _records(pipe)
    o = P._value_recursion(recs, pipe.cfg.rate)
    assert np.array_equal(pipe.pnl["value"].cpu().numpy(), o["value"])
    assert np.array_equal(pipe.pnl["turnover"].cpu().numpy()[1:], o["turnover"][1:])
    # books from the engine's predictions and tradable flags
    pred = pipe.pred.cpu().numpy()
    trad = unpack_bits(grid.tbits, pipe.T).cpu().numpy()
    rd = pipe.rdates.cpu().numpy()
    for i in np.linspace(0, pipe.nd - 1, 24).astype(int):
        t = rd[i]
        ids = np.flatnonzero(~np.isnan(pred[t]))
        L, S = P.select_books(ids, pred[t, ids], trad[t, ids], top_n)
        assert np.array_equal(recs[i]["L"], L) and np.array_equal(recs[i]["S"], S), i


def test_config_c_pooled_gram_lasso_predict(config_c):
    """Config C's regression leg at full size (41 M pooled rows x 99 columns):
    * the pooled Gram of [1, z_1..z_97, target] over train + valid (train_end twice, KKT:426-427)
      against torch fp64 D^T D of the same z-scored rows (z = (x - mu) * (1/sigma), the
      engine's zs), accumulated in 128-date chunks: rel 1e-12 of max |G|, the row count exact;
    * the Lasso (KKT:605-607) against the oracle's Gram coordinate descent
      (oracle/lasso_oracle.c, scikit-learn 1.7.2's algorithm) on the engine's Gram: coefficients
      and iteration count bit-exact, and on the reference Gram: same support, rel 1e-9;
    * lasso.predict (KKT:612) on 20 sampled test dates: b0 + sum_j b_j z_j in the engine's order
      (ascending j, zero coefficients skipped) -- bit-exact, NaN off the z-score rows."""
    import torch
    import oracle
    from afm.grid import unpack_bits
    p, grid, pipe = config_c
    sp, T, lda = pipe.sp, pipe.T, pipe.lda
    zr = unpack_bits(pipe.zrows, T)                                     # [T][lda] bool
    feat = pipe.feat.long()
    mu, rs = pipe.zs[:pipe.p, :, 0], pipe.zs[:pipe.p, :, 1]
    G = torch.zeros((pipe.p2, pipe.p2), dtype=torch.float64, device=pipe.out.device)

    def add_rows(t0, t1):
        tt, aa = torch.nonzero(zr[t0:t1], as_tuple=True)
        if len(tt) == 0:
            return torch.zeros_like(G)
        X = pipe.out[feat, t0:t1][:, tt, aa]                           # [p][n]
        Z = (X - mu[:, aa]) * rs[:, aa]
        y = pipe.out[96, t0:t1][tt, aa]
        D = torch.cat([torch.ones_like(y)[None], Z, y[None]], dim=0)
        return D @ D.T

    for t0 in range(0, sp.v1, 128):
        G += add_rows(t0, min(sp.v1, t0 + 128))
    if sp.dup:
        G += add_rows(sp.tr1 - 1, sp.tr1)
    got = pipe.pool_g[0]
    assert got[0, 0].item() == G[0, 0].item() > 4e7
    err = ((got - G).abs().max() / G.abs().max()).item()
    assert err < 1e-12, err
    # Lasso on the engine's Gram: the oracle's coordinate descent, bit for bit
    c = pipe.cfg
    n, Q, q, yy = oracle.centered_moments(got.cpu().numpy())
    w, gap, tol_y, it = oracle.lasso_gram(Q, q, yy, c.alpha * n, max_iter=c.max_iter,
                                          tol=c.lasso_tol)
    b = pipe.lasso_beta.cpu().numpy()
    assert np.array_equal(b[1:], w)
    assert int(pipe.lasso_info[2].item()) == it
    # ... and on the reference Gram: the same fit within rel 1e-9
    n2, Q2, q2, yy2 = oracle.centered_moments(G.cpu().numpy())
    w2, _, _, _ = oracle.lasso_gram(Q2, q2, yy2, c.alpha * n2, max_iter=c.max_iter, tol=c.lasso_tol)
    assert np.array_equal(w2 != 0, w != 0)
    assert np.abs(w2 - w).max() <= 1e-9 * np.abs(w).max()
    # predictions on sampled test dates
    pred = pipe.pred
    nz = np.flatnonzero(b[1:] != 0)
    for t in np.linspace(sp.s0, T - 2, 20).astype(int):
        m = zr[t]
        aa = torch.nonzero(m).flatten()
        s = torch.full((len(aa),), b[0], dtype=torch.float64, device=pred.device)
        for j in nz:
            z = (pipe.out[feat[j], t, aa] - mu[j, aa]) * rs[j, aa]
            s = s + b[1 + j] * z
        assert torch.equal(pred[t, aa], s), t
        assert torch.isnan(pred[t, ~m]).all(), t


@pytest.fixture(scope="module")
def config_b():
    return _pipeline(3000, 5040, 7)


def test_config_b_fama_macbeth_vs_oracle(config_b):
    from afm.grid import unpack_bits
    from oracle.pipeline import xs_ols
    p, grid, pipe = config_b
    pf = len(pipe.cfg.fm_features)
    assert pf == 30
    zr = unpack_bits(pipe.zrows, pipe.T).cpu().numpy()
    out = pipe.out
    fc = pipe.fm_cols.long()
    n = pipe.fm_nobs.cpu().numpy()
    fb = pipe.fm_beta.cpu().numpy()
    ok = np.flatnonzero(n > 3 * pf)
    assert len(ok) > 0.6 * pipe.T
    for t in ok[np.linspace(0, len(ok) - 1, 8).astype(int)]:
        rows = np.flatnonzero(zr[t, :grid.A])
        assert len(rows) == int(n[t])
        X = out[fc, t][:, rows].T.cpu().numpy()
        y = out[96, t][rows].cpu().numpy()
        _, B, N = xs_ols(np.zeros(len(rows), np.int64), X, y)
        err = np.abs(fb[t] - B[0]).max() / np.abs(B[0]).max()
        assert err < 1e-9, (t, err)


def test_config_b_ic_vs_oracle(config_b):
    from afm.grid import unpack_bits
    from oracle import xs as XS
    p, grid, pipe = config_b
    T, A = pipe.T, grid.A
    pred = pipe.pred.cpu().numpy()[:, :A]
    close = grid.close.cpu().numpy()[:, :A]
    pb = unpack_bits(pipe.price_bits, T).cpu().numpy()[:, :A]
    an_d = pipe.an_dates.cpu().numpy() + pipe.an_a0
    ic = pipe.an["ic"].cpu().numpy()
    picks = an_d[np.linspace(0, len(an_d) - 8, 6).astype(int)]
    t0 = int(picks.min())
    pt, pa = np.nonzero(pb[t0:])
    pt = pt + t0
    sig_t = np.concatenate([np.full(int((~np.isnan(pred[t])).sum()), t) for t in picks])
    sig_a = np.concatenate([np.flatnonzero(~np.isnan(pred[t])) for t in picks])
    date, ids, vals = XS.add_returns(sig_t, sig_a, pred[sig_t, sig_a], pt, pa, close[pt, pa])
    od, otype, oic = XS.ic_series(date, vals)
    pos = {int(t): j for j, t in enumerate(an_d)}
    types = {"return_1": 0, "return_2": 1, "return_5": 2}
    got = np.array([ic[pos[int(d)], types[str(ty)]] for d, ty in zip(od, otype)])
    assert len(got) == 3 * len(picks)
    np.testing.assert_allclose(got, oic, rtol=1e-12, atol=1e-14)


def test_config_e_bootstrap_paths_vs_oracle():
    from afm.portfolio import bootstrap_paths, bootstrap_pnl
    from oracle import portfolio as P
    p, grid, pipe = _pipeline(5000, 5040, 11)
    paths = bootstrap_paths(pipe.nd, 1024, seed=2023)
    got = bootstrap_pnl(pipe.reb, pipe.pred, pipe.rdates, paths, rate=pipe.cfg.rate)
    value = got["value"].cpu().numpy()
    assert value.shape == (1024, pipe.nd + 1) and np.isfinite(value).all()
    recs = _records(pipe)
    for j in np.linspace(0, 1023, 6).astype(int):
        o = P._value_recursion([recs[i] for i in paths[j]], pipe.cfg.rate)
        assert np.array_equal(value[j], o["value"]), j

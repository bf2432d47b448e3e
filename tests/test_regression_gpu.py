"""GPU parity of the regression kernels (R1): shifted Gram on fp64 MFMA, per-date OLS and
Fama-MacBeth vs the numpy oracle, LinearRegression drop-in vs the reference's sklearn fit.

Tolerances: rel 1e-9 (BASELINE north star) on well-conditioned designs; the Gram itself is
checked at 1e-12 relative to its scale."""
import os

import numpy as np
import pytest

from helpers import oracle_panel

pytestmark = pytest.mark.gpu

WELL = ["RSI_14", "sd_5", "corr_15", "PSY", "ROCR_20", "volsd5_15", "MACD_12_24"]


def centered_from(gram, shift):
    """(G', s) -> (n, mean[p+1], C[p+1][p+1]) on the host."""
    G = gram.cpu().numpy()
    s = shift.cpu().numpy()
    n = G[..., 0, 0]
    m = G[..., 0, 1:] / n[..., None]
    C = G[..., 1:, 1:] - G[..., 0, 1:, None] * G[..., 0, None, 1:] / n[..., None, None]
    return n, s[..., 1:] + m, C


@pytest.mark.parametrize("p,n", [(3, 5000), (30, 7000), (96, 3000), (110, 300)])
def test_gram_long_mode_vs_numpy(p, n):
    import torch
    from afm.regression import xs_gram
    rng = np.random.default_rng(p)
    X = rng.normal(size=(n, p + 1)) * rng.uniform(0.1, 1e3, size=p + 1) + rng.normal(size=p + 1) * 50
    X[rng.random(n) < 0.01, rng.integers(0, p + 1)] = np.nan      # dropped rows
    X[5, 0] = np.inf
    Z = torch.from_numpy(np.ascontiguousarray(X.T)).cuda()
    L = 1000
    nseg = (n + L - 1) // L
    gram, shift = xs_gram(Z, n, L, L, list(range(p)), p, nseg=nseg, row_limit=n)
    nn, mean, C = centered_from(gram, shift)
    for s in range(nseg):
        blk = X[s * L:(s + 1) * L]
        blk = blk[np.isfinite(blk).all(axis=1)]
        assert nn[s] == len(blk)
        assert np.allclose(mean[s], blk.mean(axis=0), rtol=1e-12, atol=0)
        ref = (blk - blk.mean(0)).T @ (blk - blk.mean(0))
        scale = np.sqrt(np.outer(np.diag(ref), np.diag(ref)))
        assert np.abs(C[s] - ref).max() / scale.max() < 1e-12


@pytest.mark.parametrize("mode", ["grid", "long"])
def test_gram_fast_pass_identical_to_checked(mode, monkeypatch):
    """FAST staging + REDO of segments with a non-finite diagonal == checked staging, bit for bit
    (segments with masked-in non-finite rows in both x and y, and clean segments)."""
    import torch
    from afm.grid import pack_bits
    from afm.regression import xs_gram
    rng = np.random.default_rng(9)
    p, T, lda = 40, 24, 640
    Z = torch.from_numpy(rng.normal(size=(p + 1, T, lda)) * 3 + 20).cuda()
    Z[3, 2, 17] = float("inf")
    Z[p, 5, 100] = float("nan")                      # y
    Z[7, 9, 0] = float("nan")                        # the would-be shift row
    Z[0, 11, 33:40] = float("-inf")
    valid = torch.from_numpy(rng.random((T, lda)) < 0.9).cuda()
    bits = pack_bits(valid)
    if mode == "grid":
        args = (Z, T * lda, lda, lda, list(range(p)), p)
        kw = dict(bits=bits, nseg=T)
    else:
        flat = Z.reshape(p + 1, T * lda)
        args = (flat, T * lda, 500, 500, list(range(p)), p)
        kw = dict(nseg=(T * lda + 499) // 500, row_limit=T * lda - 77)
    g1, s1 = xs_gram(*args, **kw)
    from afm import _lib
    with _lib.options(gram_checked=1):
        g0, s0 = xs_gram(*args, **kw)
    torch.cuda.synchronize()
    assert torch.equal(s0, s1)
    assert torch.equal(g0, g1)
    assert torch.isfinite(g0).all()


def _panel_rows(seed=3, A=200, T=400):
    from afm.synthetic import make_panel
    p = make_panel(A, T, seed=seed, hole_frac=0.003)
    tt, aa, fac = oracle_panel(p)
    return p, tt, aa, fac


def test_cross_sectional_ols_vs_oracle():
    import torch
    import afm
    from afm.regression import cross_sectional_ols
    from oracle import pipeline as PL
    p, tt, aa, fac = _panel_rows()
    grid = afm.PanelGrid.from_panel(p)
    out, nanfree = afm.factor_panel(grid)
    cols = [afm.FACTOR_NAMES.index(c) for c in WELL]
    t0 = 60
    res = cross_sectional_ols(out, nanfree, grid.lda, cols, t0=t0, A=grid.A)
    beta = res["beta"].cpu().numpy()
    nobs = res["nobs"].cpu().numpy()
    # oracle: rows surviving dropna (96 factors + target finite), finite selected columns
    X, y = fac[:, cols], fac[:, 96]
    use = (~np.isnan(fac[:, :96]).any(axis=1)) & np.isfinite(y) & np.isfinite(X).all(axis=1)
    use &= tt >= t0
    d, B, N = PL.xs_ols(tt[use], X[use], y[use])
    assert np.array_equal(nobs[d - t0], N)
    got = beta[d - t0]
    err = np.abs(got - B).max(axis=1) / np.abs(B).max(axis=1)
    assert err.max() < 1e-9, err.max()
    m, t = afm.regression.fama_macbeth(res["beta"], res["rank"])
    ok = res["rank"].cpu().numpy() > 0
    bm = beta[ok]
    assert np.allclose(m.cpu().numpy(), bm.mean(0), rtol=1e-10)
    tref = bm.mean(0) / (bm.std(0, ddof=1) / np.sqrt(len(bm)))
    assert np.allclose(t.cpu().numpy(), tref, rtol=1e-9)
    torch.cuda.synchronize()


def test_linear_regression_dropin_matches_reference(golden_dir):
    """afm.LinearRegression on the notebook's z-scored train+valid design (KKT:582-590)."""
    import pandas as pd
    import oracle
    from afm.regression import LinearRegression
    from oracle import pipeline as PL
    g = np.load(os.path.join(golden_dir, "factors_pipeline.npz"))
    df = pd.DataFrame({
        "data_date": g["in_date"].astype("datetime64[ns]"), "security_id": g["in_id"],
        "close_price": g["in_close"], "volume": g["in_volume"], "ret1d": g["in_ret1d"],
        "excess_ret1d": g["in_excess"], "group_id": g["in_group"],
        "in_trading_universe": np.where(g["in_tradable"], "Y", "N")})
    out = oracle.compute_factors(df).sort_values(["data_date", "security_id"])
    cols = PL.feature_columns(out.columns.drop(["data_date", "security_id"]))
    d = out["data_date"].values.astype("datetime64[ns]").astype(np.int64)
    ids = out["security_id"].values
    X, y = out[cols].to_numpy(np.float64), out["target"].to_numpy()
    uid = np.unique(ids)
    tr, va, te = PL.split_masks(d)
    mu, sd = PL.group_stats(ids[tr], X[tr], uid)
    parts = {}
    for nm, m in (("tr", tr), ("va", va), ("te", te)):
        zz, keep = PL.zscore(ids[m], X[m], uid, mu, sd)
        parts[nm] = (zz[keep], y[m][keep])
    o = np.load(os.path.join(golden_dir, "ols_pipeline.npz"))
    sub = [cols.index(c) for c in o["sub_cols"]]
    Xtr = pd.DataFrame(np.vstack([parts["tr"][0], parts["va"][0]])[:, sub], columns=list(o["sub_cols"]))
    ytr = pd.DataFrame({"target": np.r_[parts["tr"][1], parts["va"][1]]})
    m = LinearRegression().fit(Xtr, ytr)
    assert m.coef_.shape == (1, len(sub)) and m.intercept_.shape == (1,)
    ref = np.r_[o["sub_intercept"], o["sub_coef"]]
    got = np.r_[m.intercept_, m.coef_.ravel()]
    assert np.abs(got - ref).max() / np.abs(ref).max() < 1e-9
    pred = m.predict(pd.DataFrame(parts["te"][0][:, sub], columns=list(o["sub_cols"])))
    assert pred.shape == (len(parts["te"][0]), 1)
    assert np.abs(pred.ravel() - o["sub_pred"]).max() / np.abs(o["sub_pred"]).max() < 1e-9
    # the notebook's full 97-column design (near-collinear): predictions agree to 1e-6
    Xf = np.vstack([parts["tr"][0], parts["va"][0]])
    mf = LinearRegression().fit(Xf, ytr["target"].to_numpy())
    pf = mf.predict(parts["te"][0])
    assert np.abs(pf - o["full_pred"]).max() / np.abs(o["full_pred"]).max() < 1e-6


@pytest.mark.parametrize("p,nseg,cut", [(96, 4032, 2048), (7, 700, 320), (30, 50, 0), (5, 1, 0)])
def test_pool_tree_split_identical(p, nseg, cut):
    """afm_pool_moments_f64's fixed tree == the multi-GPU composition (each 64-aligned date range
    through levels 0-1 with afm_pool_segments_f64 per 16 then 4, the 64-date blocks of both ranges
    through afm_pool_tree_f64 from level 2): bit-identical; and the pooled moments match the
    exact centered sums of all segments (rel 1e-12)."""
    import torch
    from afm import _lib
    L, P = _lib.lib(), _lib.ptr
    rng = np.random.default_rng(nseg + p)
    p2 = p + 2
    dev = torch.device("cuda:0")
    # per-segment shifted moments of random rows: G = [n, sum(z - s); ..., sum (z-s)(z-s)']
    n = rng.integers(0, 40, size=nseg).astype(np.float64)
    n[rng.random(nseg) < 0.05] = 0                       # empty segments are skipped
    G = np.zeros((nseg, p2, p2))
    S = np.zeros((nseg, p2))
    allz = []
    for k in range(nseg):
        z = rng.normal(3.0, 2.0, size=(int(n[k]), p + 1))
        allz.append(z)
        s = z[0] if len(z) else np.zeros(p + 1)
        d = z - s
        G[k, 0, 0] = n[k]
        G[k, 0, 1:] = G[k, 1:, 0] = d.sum(axis=0)
        G[k, 1:, 1:] = d.T @ d
        S[k, 1:] = s
    g = torch.from_numpy(G).to(dev)
    sh = torch.from_numpy(S).to(dev)
    ctx = _lib.Context.get(0)
    h = ctx.bind_stream()
    og = torch.empty((1, p2, p2), dtype=torch.float64, device=dev)
    osh = torch.empty((1, p2), dtype=torch.float64, device=dev)
    _lib.check(L.afm_pool_moments_f64(h, P(g), P(sh), p, nseg, P(og), P(osh)), "pool")
    blocks_g, blocks_s = [], []
    for lo, hi in ((0, cut), (cut, nseg)):
        m = hi - lo
        if m == 0:
            continue
        n16, n64 = (m + 15) // 16, (m + 63) // 64
        g16 = torch.empty((n16, p2, p2), dtype=torch.float64, device=dev)
        s16 = torch.empty((n16, p2), dtype=torch.float64, device=dev)
        g64 = torch.empty((n64, p2, p2), dtype=torch.float64, device=dev)
        s64 = torch.empty((n64, p2), dtype=torch.float64, device=dev)
        _lib.check(L.afm_pool_segments_f64(h, P(g[lo:hi]), P(sh[lo:hi]), p, m, 16, P(g16),
                                           P(s16)), "level 0")
        _lib.check(L.afm_pool_segments_f64(h, P(g16), P(s16), p, n16, 4, P(g64), P(s64)),
                   "level 1")
        blocks_g.append(g64)
        blocks_s.append(s64)
    bg = torch.cat(blocks_g).contiguous()
    bs = torch.cat(blocks_s).contiguous()
    tg = torch.empty_like(og)
    ts = torch.empty_like(osh)
    _lib.check(L.afm_pool_tree_f64(h, P(bg), P(bs), p, bg.shape[0], 2, P(tg), P(ts)), "tree")
    torch.cuda.synchronize()
    assert torch.equal(og, tg) and torch.equal(osh, ts)
    z = np.concatenate(allz)
    mu = z.mean(axis=0)
    C = (z - mu).T @ (z - mu)
    got = og[0].cpu().numpy()
    assert got[0, 0] == len(z)
    assert np.abs(osh[0, 1:].cpu().numpy() - mu).max() <= 1e-12 * np.abs(mu).max()
    assert np.abs(got[1:, 1:] - C).max() <= 1e-12 * np.abs(C).max()

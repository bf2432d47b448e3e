"""GPU parity of the signal-evaluation path (A1-A4): the AlphaSignalAnalyzer drop-in against the
reference's own outputs (tests/golden/analyzer_*.npz), bit-exact."""
import os

import numpy as np
import pandas as pd
import pytest

from helpers import same

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,fname", [("zfactor", "RSI_14"), ("lrpred", "lr_predict")])
def test_analyzer_matches_reference(golden_dir, name, fname):
    from afm.analyzer import AlphaSignalAnalyzer
    g = np.load(os.path.join(golden_dir, f"analyzer_{name}.npz"))
    sig = pd.DataFrame({fname: g["sig_val"]}, index=pd.MultiIndex.from_arrays(
        [g["sig_date"].astype("datetime64[ns]"), g["sig_id"]]))
    px = pd.DataFrame({"close_price": g["px_close"]}, index=pd.MultiIndex.from_arrays(
        [g["px_date"].astype("datetime64[ns]"), g["px_id"]]))
    an = AlphaSignalAnalyzer(sig, fname, px)
    an.run()
    fd = an.factor_df
    assert same(fd.index.get_level_values(0).values.astype(np.int64), g["fr_date"])
    assert same(fd.index.get_level_values(1).values, g["fr_id"])
    assert same(fd.to_numpy(np.float64), g["fr_vals"])
    assert same(an.ic_df["date"].values.astype(np.int64), g["ic_date"])
    assert list(an.ic_df["Type"]) == list(g["ic_type"])
    assert same(an.ic_df["IC"].values, g["ic"])
    assert same(an.ir_df["year"].values, g["ir_year"]) and list(an.ir_df["Type"]) == list(g["ir_type"])
    assert same(an.ir_df["IR"].values, g["ir"])
    for rt in ("return_1", "return_2", "return_5"):
        ld = an.layered_ret_dfs[rt]
        assert same(ld["date"].values.astype(np.int64), g[f"lay_{rt}_date"])
        assert same(ld["layer"].values, g[f"lay_{rt}_layer"])
        assert same(ld[rt].values, g[f"lay_{rt}"]), rt
        ls = an.ls_ret_dfs[rt]
        assert same(ls["date"].values.astype(np.int64), g[f"ls_{rt}_date"])
        assert same(ls["layer"].values, g[f"ls_{rt}_layer"])
        assert same(ls[rt].values, g[f"ls_{rt}"]), rt
    assert same(an.port_ret_df["date"].values.astype(np.int64), g["pt_date"])
    assert list(an.port_ret_df["Type"]) == list(g["pt_type"])
    assert same(an.port_ret_df["Returns"].values, g["pt_ret"])


def test_analyzer_large_panel_vs_oracle():
    """Dates with > 2048 rows (multi-chunk ranks, multi-leaf pairwise sums) vs the oracle."""
    from afm.analyzer import AlphaSignalAnalyzer
    from oracle import xs
    rng = np.random.default_rng(9)
    T, A = 12, 5000
    dates = np.asarray(np.busday_offset(np.datetime64("2017-03-01"), np.arange(T), roll="forward"),
                       dtype="datetime64[ns]")
    tt, aa = np.nonzero(rng.random((T, A)) < 0.97)
    d, i = dates[tt], 100 + aa
    close = 30 * np.exp(rng.normal(0, 0.05, len(tt)))
    v = np.round(rng.normal(size=len(tt)), 3)          # many exact ties in the signal
    keep = rng.random(len(tt)) < 0.95
    sig = pd.DataFrame({"f": v[keep]}, index=pd.MultiIndex.from_arrays([d[keep], i[keep]]))
    px = pd.DataFrame({"close_price": close}, index=pd.MultiIndex.from_arrays([d, i]))
    an = AlphaSignalAnalyzer(sig, "f", px)
    an.run()
    o = xs.analyze(d[keep].astype(np.int64), i[keep], v[keep], d.astype(np.int64), i, close)
    assert same(an.factor_df.to_numpy(np.float64), o["fr_vals"])
    assert same(an.ic_df["IC"].values, o["ic"])
    for rt in ("return_1", "return_2", "return_5"):
        assert same(an.layered_ret_dfs[rt][rt].values, o[f"lay_{rt}"])
        assert same(an.ls_ret_dfs[rt][rt].values, o[f"ls_{rt}"])
    assert same(an.port_ret_df["Returns"].values, o["pt_ret"])


@pytest.mark.parametrize("lda,kind", [(64, "normal"), (1024, "ties"), (12288, "normal"),
                                      (12288, "ties"), (12352, "normal")])
def test_layers_match_exact_ranks(lda, kind):
    """afm_xs_layers_f64 (no sort) gives xs_stats exactly what it reads of afm_xs_rank_f64's ranks:
    each row's decile layer (KKT:328-330) and the descending ranks 1..10 (KKT:359-369), with
    method='first' ties; row counts 0, 1, 9, 10, 11, ... up to the register capacity (12288) and
    past it (the sorting fallback)."""
    import torch
    from afm import _lib
    rng = np.random.default_rng(lda)
    T = 40
    counts = np.concatenate([[0, 1, 2, 9, 10, 11, 19, 20, 21, lda],
                             rng.integers(0, lda + 1, T - 10)]).astype(np.int32)
    if kind == "ties":
        v = rng.integers(-3, 4, (T, lda)).astype(np.float64) * 0.25
        v[::3] = 1.5                                       # all-equal dates
        v[1::7, ::5] = -0.0                                # signed zeros tie with 0
    else:
        v = rng.normal(size=(T, lda))
    dev = torch.device("cuda", 0)
    rows = torch.from_numpy(v).to(dev)
    nrows = torch.from_numpy(counts).to(dev)
    L, P, h = _lib.lib(), _lib.ptr, _lib.Context.get(0).bind_stream()
    out = []
    for fn in (L.afm_xs_rank_f64, L.afm_xs_layers_f64):
        skey = torch.empty((T, lda), dtype=torch.int64, device=dev)
        sidx = torch.empty((T, lda), dtype=torch.int32, device=dev)
        ra = torch.full((T, lda), -1, dtype=torch.int32, device=dev)
        rd = torch.full((T, lda), -1, dtype=torch.int32, device=dev)
        _lib.check(fn(h, T, lda, P(rows), P(nrows), P(skey), P(sidx), P(ra), P(rd)), "rank")
        out.append((ra.cpu().numpy(), rd.cpu().numpy()))
    (ra0, rd0), (ra1, rd1) = out
    for t in range(T):
        n = int(counts[t])
        if n == 0:
            continue
        lay0 = np.minimum((ra0[t, :n] / n * 10).astype(int) + 1, 10)
        lay1 = np.minimum((ra1[t, :n] / n * 10).astype(int) + 1, 10)
        assert np.array_equal(lay0, lay1), t
        top0 = np.where(rd0[t, :n] <= 10, rd0[t, :n], n + 1)
        if lda <= 12288:
            assert np.array_equal(top0, rd1[t, :n]), t
        else:                                              # the fallback: exact ranks
            assert np.array_equal(rd0[t, :n], rd1[t, :n]), t

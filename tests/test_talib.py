"""talib factor variant (KKT:176-270).  TA-Lib is absent here and the
reference ships no TA-Lib outputs, so parity with TA-Lib itself is UNPINNED: the CPU tests pin
the restatement (oracle/talib_oracle.c) to known answers that follow from TA-Lib's documented
lookbacks and seeds; the GPU tests hold the HIP kernel bit-exact to that restatement and the
drop-in frame to the oracle-assembled one (shared columns from the pinned No-talib oracle)."""
import numpy as np
import pytest

from helpers import mismatch_report, panel_long, same

CASES = [(70, 333, 1, dict(edge_cases=True, hole_frac=0.02, listing_frac=0.3)),
         (130, 700, 2, dict(hole_frac=0.002))]


def _series(x, v=None):
    import oracle
    v = np.full(len(x), 10.0) if v is None else v
    return oracle.talib_factors_long(np.array([0, len(x)]), np.asarray(x, float), v)


def test_known_answers_lookbacks_and_seeds():
    x = np.arange(1.0, 101.0)
    o = _series(x)
    assert np.isnan(o[:5, 0]).all() and o[5, 0] == 3.5            # SMA_6: first at index 5
    assert o[5, 12] == 3.5 and o[6, 12] == 4.5                      # EMA_6 seeded by the SMA
    assert o[5, 24] == 35.0                                         # VSMA_6 = SMA(volume*close)
    assert np.isnan(o[:13, 37]).all() and o[13, 37] == 7.5         # BBANDS_middle_14
    assert np.isclose((o[13, 36] - o[13, 37]) / 2, np.std(x[:14]), rtol=1e-12)   # ddof = 0
    for j, slow in enumerate((18, 24, 30)):                        # MACD: slow - 1 + 8
        assert np.flatnonzero(~np.isnan(o[:, 60 + j]))[0] == slow + 7
    for j, n in enumerate((8, 14, 20)):                            # RSI: first at n, 100 if rising
        assert np.flatnonzero(~np.isnan(o[:, 63 + j]))[0] == n
        assert o[n, 63 + j] == 100.0
    assert np.isnan(o[0, 66]) and o[1, 66] == 10.0                  # PVT: no cumsum
    assert list(o[:3, 67]) == [10.0, 20.0, 30.0]                    # OBV starts at volume[0]


def test_constant_and_flat_series():
    o = _series(np.full(80, 42.0), np.arange(1.0, 81.0))
    ok = ~np.isnan(o[:, 36])
    assert (o[ok, 36] == o[ok, 37]).all() and (o[ok, 38] == o[ok, 37]).all()   # sd = 0
    assert (o[~np.isnan(o[:, 60]), 60] == 0.0).all()                 # MACD of a constant
    assert (o[~np.isnan(o[:, 63]), 63] == 0.0).all()                 # |gain + loss| < 1e-8
    assert (o[:, 67] == 1.0).all()                                   # equal closes: unchanged
    assert (o[~np.isnan(o[:, 12]), 12] == 42.0).all()


def test_short_series_all_nan():
    o = _series(np.linspace(1, 2, 5))
    assert np.isnan(o[:, :66]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("A,T,seed,kw", CASES)
def test_talib_kernel_vs_oracle(A, T, seed, kw):
    import torch
    import afm
    import oracle
    from afm.synthetic import make_panel
    from afm.talib_factors import talib_panel, _TL
    p = make_panel(A, T, seed=seed, **kw)
    grid = afm.PanelGrid.from_panel(p)
    out = talib_panel(grid)
    tt, aa, off = panel_long(p)
    ref = oracle.talib_factors_long(off, p.close[tt, aa], p.volume[tt, aa])
    got = out[:, torch.from_numpy(tt).cuda(), torch.from_numpy(aa).cuda()].T.cpu().numpy()
    assert same(got, ref), mismatch_report(got, ref, _TL)


@pytest.mark.gpu
def test_compute_factors_talib_dropin():
    import pandas as pd
    import oracle
    from afm.synthetic import make_panel, to_frame
    from afm.talib_factors import TALIB_NAMES, TALIB_PLANE, compute_factors_talib
    p = make_panel(40, 300, seed=4, edge_cases=True, hole_frac=0.01)
    df = to_frame(p)
    got = compute_factors_talib(df)
    # oracle frame: per-security rows, shared columns from the pinned No-talib oracle
    d = df.sort_values(by=["security_id", "data_date"]).reset_index(drop=True)
    sid = d["security_id"].to_numpy()
    off = np.r_[np.flatnonzero(np.r_[True, sid[1:] != sid[:-1]]), len(sid)].astype(np.int64)
    c, v = d["close_price"].to_numpy(), d["volume"].to_numpy()
    fac = oracle.factors_long(off, c, v, d["ret1d"].to_numpy(), d["excess_ret1d"].to_numpy())
    tl = oracle.talib_factors_long(off, c, v)
    cols = [tl[:, TALIB_PLANE[n]] if n in TALIB_PLANE else fac[:, oracle.FACTOR_NAMES.index(n)]
            for n in TALIB_NAMES]
    want = pd.concat([d, pd.DataFrame(np.stack(cols, 1), columns=TALIB_NAMES)], axis=1).dropna()
    assert list(got.columns) == list(want.columns)
    assert np.array_equal(got.index.values, want.index.values)
    assert same(got[TALIB_NAMES].to_numpy(), want[TALIB_NAMES].to_numpy())

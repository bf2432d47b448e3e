"""GPU parity of the factor panel (afm_factors_f64) -- bit-exact against the oracle and the
reference's own outputs (tests/golden/factors_*.npz)."""
import os

import numpy as np
import pandas as pd
import pytest

from helpers import mismatch_report, oracle_panel, same

pytestmark = pytest.mark.gpu


def frame_from(g):
    return pd.DataFrame({
        "data_date": g["in_date"].astype("datetime64[ns]"), "security_id": g["in_id"],
        "close_price": g["in_close"], "volume": g["in_volume"], "ret1d": g["in_ret1d"],
        "excess_ret1d": g["in_excess"], "group_id": g["in_group"],
        "in_trading_universe": np.where(g["in_tradable"], "Y", "N")})


@pytest.mark.parametrize("name", ["edge", "scales", "pipeline"])
def test_compute_factors_matches_reference(golden_dir, name):
    import afm
    g = np.load(os.path.join(golden_dir, f"factors_{name}.npz"))
    out = afm.compute_factors(frame_from(g))
    assert np.array_equal(out.index.values, g["out_index"])
    assert np.array_equal(out["security_id"].values, g["out_id"])
    cols = list(g["out_cols"])
    got = out[cols].to_numpy(np.float64)
    assert same(got, g["out"]), mismatch_report(got, g["out"], cols)


@pytest.mark.parametrize("A,T,seed,kw", [
    (70, 333, 1, dict(edge_cases=True, hole_frac=0.02, listing_frac=0.3)),
    (300, 900, 2, dict(hole_frac=0.002)),
    (64, 64, 3, dict(hole_frac=0.05)),
    (5, 130, 4, dict(edge_cases=True)),
])
def test_factor_grid_vs_oracle(A, T, seed, kw):
    import torch
    import afm
    from afm.synthetic import make_panel
    p = make_panel(A, T, seed=seed, **kw)
    grid = afm.PanelGrid.from_panel(p)
    out, nanfree = afm.factor_panel(grid)
    torch.cuda.synchronize()
    tt, aa, ref = oracle_panel(p)
    got = out[:, torch.from_numpy(tt).cuda(), torch.from_numpy(aa).cuda()].T.cpu().numpy()
    assert same(got, ref), mismatch_report(got, ref, afm.FACTOR_NAMES)
    # absent cells untouched (still the NaN fill), nanfree = present & no NaN in 96 factors
    o = out.cpu().numpy()
    assert np.isnan(o[:, ~p.valid]).all()
    nf = afm.unpack_bits(nanfree, T).cpu().numpy()
    exp = np.zeros_like(p.valid)
    exp[tt, aa] = ~np.isnan(ref[:, :96]).any(axis=1)
    assert np.array_equal(nf, exp)


@pytest.mark.parametrize("types,pair,A", [("1", "1", 200), ("3", "1", 200), ("3", "1", 300),
                                          ("3", "0", 200), ("5", "1", 200), ("15", "1", 200),
                                          ("110", "0", 200), ("106", "0", 300), ("105", "0", 200),
                                          ("103", "0", 300), ("206", "0", 300), ("206", "0", 200)])
def test_factor_workgroup_splits_identical(types, pair, A, monkeypatch):
    """Every launch shape gives the same bit-exact panel and masks: the 15-set partition split
    over 1, 3, 5 or 15 workgroups per block (paired two items per workgroup or not, factor_pair;
    A = 300 leaves the last pair half idle), and the 30-set small-grid partition (split
    correlations, return rings) over 10, 6, 5 or 3 workgroups per block (codes 110 / 106 / 105 /
    103: 3, 5, 6, 10 job waves each), and the 60-set partition (split correlations and sd ratios)
    over 6 workgroups of 10 job waves (code 206).  The shape is chosen from the shard's block
    count; the context option factor_split overrides."""
    import torch
    import afm
    from afm.synthetic import make_panel
    p = make_panel(A, 500, seed=9, edge_cases=True, hole_frac=0.01, listing_frac=0.2)
    grid = afm.PanelGrid.from_panel(p)
    from afm import _lib
    fin = torch.zeros_like(grid.vbits)
    with _lib.options(factor_split=int(types), factor_pair=int(pair)):
        out, nanfree = afm.factor_panel(grid, finite=fin)
    torch.cuda.synchronize()
    tt, aa, ref = oracle_panel(p)
    got = out[:, torch.from_numpy(tt).cuda(), torch.from_numpy(aa).cuda()].T.cpu().numpy()
    assert same(got, ref), mismatch_report(got, ref, afm.FACTOR_NAMES)
    nf = afm.unpack_bits(nanfree, p.T).cpu().numpy()
    ff = afm.unpack_bits(fin, p.T).cpu().numpy()
    exp_n = np.zeros_like(p.valid)
    exp_n[tt, aa] = ~np.isnan(ref[:, :96]).any(axis=1)
    exp_f = np.zeros_like(p.valid)
    exp_f[tt, aa] = np.isfinite(ref[:, :96]).all(axis=1)
    assert np.array_equal(nf, exp_n) and np.array_equal(ff, exp_f)


def test_factor_kernel_rejects_bad_shapes():
    import torch
    import afm
    from afm import _lib
    from afm.synthetic import make_panel
    p = make_panel(10, 100, seed=0)
    grid = afm.PanelGrid.from_panel(p)
    ctx = _lib.Context.get()
    rc = _lib.lib().afm_factors_f64(ctx.bind_stream(), 100, 10, 60, *([None] * 8))
    assert rc != 0 and b"lda" in _lib.lib().afm_last_error()
    torch.cuda.synchronize()


@pytest.mark.parametrize("split", [0, 3])
def test_clean_fast_step_matches_general_step(monkeypatch, split):
    """The clean-window fast step (factors.hip kClean) and the general step give the same
    bit-exact panel, with same-value runs, zero volumes and NaN closes planted inside otherwise
    clean stretches (each forces the general step for ~58 observations, then the fast step
    resumes on the carried states) -- in the small-grid partition (auto at 256 assets) and the
    15-set one (split 3)."""
    import torch
    import afm
    from afm.synthetic import make_panel
    p = make_panel(256, 700, seed=11, hole_frac=0.01, listing_frac=0.2)
    rng = np.random.default_rng(5)
    for a in rng.choice(256, 40, replace=False):          # flat runs: the same-value rules
        t0, n = int(rng.integers(100, 600)), int(rng.integers(3, 70))
        p.close[t0:t0 + n, a] = p.close[t0, a]
    for a in rng.choice(256, 10, replace=False):
        p.volume[int(rng.integers(100, 690)), a] = 0.0
    for a in rng.choice(256, 6, replace=False):
        p.close[int(rng.integers(100, 690)), a] = np.nan
    grid = afm.PanelGrid.from_panel(p)
    outs = {}
    from afm import _lib
    for flag in ("1", "0"):
        fin = torch.zeros_like(grid.vbits)
        with _lib.options(factor_fast=int(flag == "0"), factor_split=split):
            out, nanfree = afm.factor_panel(grid, finite=fin)
        torch.cuda.synchronize()
        outs[flag] = (out.clone(), nanfree.clone(), fin.clone())
    assert torch.equal(outs["1"][1], outs["0"][1]) and torch.equal(outs["1"][2], outs["0"][2])
    a, b = outs["1"][0], outs["0"][0]
    assert torch.equal(a.isnan(), b.isnan()) and torch.equal(a.nan_to_num(0.0), b.nan_to_num(0.0))
    assert torch.equal(a.signbit() & ~a.isnan(), b.signbit() & ~b.isnan())      # -0 vs +0 too
    tt, aa, ref = oracle_panel(p)
    got = b[:, torch.from_numpy(tt).cuda(), torch.from_numpy(aa).cuda()].T.cpu().numpy()
    assert same(got, ref), mismatch_report(got, ref, afm.FACTOR_NAMES)


@pytest.mark.parametrize("split", [0, 110, 3])
def test_factor_range_part_and_masks_identical(split):
    """afm_factors_range_part_f64 (mask partials to a caller buffer, no labels) slab by slab with
    afm_factor_masks_f64 run afterwards equals one afm_factors_f64 call: panel columns 0-95 and
    both row masks, bit for bit."""
    import torch
    import afm
    from afm import _lib
    from afm.synthetic import make_panel
    L, P, chk = _lib.lib(), _lib.ptr, _lib.check
    p = make_panel(300, 450, seed=21, edge_cases=True, hole_frac=0.01, listing_frac=0.2)
    grid = afm.PanelGrid.from_panel(p)
    with _lib.options(factor_split=split) as ctx:
        fin = torch.zeros_like(grid.vbits)
        out, nanfree = afm.factor_panel(grid, finite=fin)
        T, A, lda = p.T, p.A, grid.lda
        h = ctx.bind_stream()
        out2 = torch.full_like(out, float("nan"))
        nf2, fin2 = torch.zeros_like(nanfree), torch.zeros_like(fin)
        st = torch.empty(int(L.afm_factors_state_bytes(ctx.handle, A)) // 8 + 1,
                         dtype=torch.float64, device="cuda")
        for t0, t1 in ((0, 128), (128, 320), (320, T)):
            part = torch.empty(int(L.afm_factors_part_words(ctx.handle, A, lda, t0, t1)),
                               dtype=torch.int64, device="cuda")
            chk(L.afm_factors_range_part_f64(h, T, A, lda, t0, t1, P(grid.close), P(grid.volume),
                                             P(grid.vbits), P(out2), P(st), P(part)), "slab")
            chk(L.afm_factor_masks_f64(h, T, A, lda, t0, t1, P(grid.vbits), P(part), P(nf2),
                                       P(fin2)), "masks")
        torch.cuda.synchronize()
    assert torch.equal(out[:96].view(torch.int64), out2[:96].view(torch.int64))
    assert torch.equal(nanfree, nf2) and torch.equal(fin, fin2)

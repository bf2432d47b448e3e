"""Secondary measurements beside bench.py's headline step (one JSON line per stage):

* zscore    -- per-security z-score (KKT:446-451) of the 97 feature planes of the config-C panel:
               train-window stats pass + in-place apply pass (HBM-bound; algorithmic bytes
               8 B per (column, train row) + 16 B per (column, applied row)).
* bootstrap -- BASELINE config E: 1,024 bootstrap paths x 5,000 assets: rebalance (books,
               rolling-252 covariance, exact KKT weights) once per date, then every path's
               union alignment, turnover DAGs and value recursion.
* lasso     -- KKT:605-607 on the config-C pooled train+valid moments (96 factors, ~38 M rows):
               afm_lasso_cd_f64 with the reference's alpha=2e-4, max_iter=10000, tol=1e-4.
* ingest    -- merge_datasets' fill steps (KKT:145-161) at config-C scale: 3 value columns on a
               10,000 x 5,040 union grid (ffill per security + per-date pairwise mean fill) and
               the per-date excess-return demean over 47.9 M reference rows.
* talib     -- the 68 TA-Lib columns of the talib variant (KKT:176-270) on the config-C panel;
               algorithmic bytes 16 read + 68 x 8 written per present asset-day.
* intraday  -- BASELINE config D: 3,000 assets x 196,560 one-minute bars (2 years x 252 days x
               390 bars), the 98-column factor build streamed over asset groups sized to HBM
               (afm/intraday.py); algorithmic bytes 816 per present asset-bar.
Usage: python tools/extra_bench.py [--only zscore|bootstrap|lasso|ingest|talib|intraday] [--reps N]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alpha-multi-factor-models_amd")]


def timed(fn, reps):
    import torch
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def bench_zscore(reps):
    import torch
    import afm
    from afm.factors import N_FACTORS, TARGET
    from afm.synthetic import make_panel
    from afm.zscore import zscore_grid
    A, T = 10000, 5040
    grid = afm.PanelGrid.from_panel(make_panel(A, T, seed=2023))
    out, nanfree = afm.factor_panel(grid)
    cols = [c for c in range(N_FACTORS) if c != TARGET]            # 96 factors + tmr_ret1d
    t_tr = int(T * 0.6)
    rows_tr = int(afm.unpack_bits(nanfree, T)[:t_tr].sum().item())
    rows = int(afm.unpack_bits(nanfree, T).sum().item())
    ms = timed(lambda: zscore_grid(out, grid.lda, cols, nanfree, train=(0, t_tr)), reps)
    K = len(cols)
    byts = 8 * K * rows_tr + 16 * K * rows
    return {"stage": "zscore", "workload": f"{A} assets x {T} days, {K} columns, train {t_tr} dates",
            "ms": round(ms, 3), "algorithmic_GB": round(byts / 1e9, 2),
            "GBps": round(byts / (ms * 1e-3) / 1e9, 1)}


def bench_bootstrap(reps, n_paths=1024, A=5000, T=5040):
    import numpy as np
    import torch
    import afm
    from afm.portfolio import bootstrap_paths, bootstrap_pnl, rebalance
    from afm.synthetic import make_panel
    g = afm.PanelGrid.from_panel(make_panel(A, T, seed=2023))
    t_test = int(T * 0.8)
    rng = np.random.default_rng(7)
    pred = torch.from_numpy(rng.normal(size=(T, g.lda))).cuda()
    pred[:t_test] = float("nan")
    pred[~g.valid] = float("nan")
    dates = torch.arange(t_test, T - 1, dtype=torch.int32, device="cuda")
    nd = int(dates.numel())
    reb = {}

    def run_reb():
        reb.update(rebalance(pred, g.tbits, g.ret1d, g.vbits, g.close, g.ret1d, dates, A=A,
                             top_n=10, window=252))
    ms_reb = timed(run_reb, reps)
    paths = torch.from_numpy(bootstrap_paths(nd, n_paths, seed=2023)).cuda()
    ms_boot = timed(lambda: bootstrap_pnl(reb, pred, dates, paths), reps)
    return {"stage": "bootstrap", "workload": f"config E: {n_paths} paths x {nd} rebalance dates, "
                                              f"{A} assets, rolling-252 cov + exact KKT top/bottom-10",
            "rebalance_ms": round(ms_reb, 3), "paths_ms": round(ms_boot, 3),
            "path_steps_per_s": round(n_paths * nd / ((ms_boot) * 1e-3), 1)}


def bench_lasso(reps):
    import torch
    import afm
    from afm import _lib
    from afm.pipeline import Pipeline
    from afm.synthetic import make_panel
    A, T = 10000, 5040
    pipe = Pipeline(afm.PanelGrid.from_panel(make_panel(A, T, seed=2023)))
    pipe.step()
    torch.cuda.synchronize()
    p = pipe.p
    n = float(pipe.pool_g[0, 0, 0].item())
    w = torch.empty(p, dtype=torch.float64, device="cuda")
    info = torch.empty(3, dtype=torch.float64, device="cuda")
    h = _lib.Context.get(0).bind_stream()

    def run():
        _lib.check(_lib.lib().afm_lasso_cd_f64(h, _lib.ptr(pipe.pool_g), p, 2e-4 * n, 0.0, 10000,
                                               1e-4, 0, _lib.ptr(w), _lib.ptr(info)))
    ms = timed(run, reps)
    gap, tol_y, it = info.cpu().numpy()
    return {"stage": "lasso", "workload": f"config C pooled moments: {int(n)} rows x {p} factors, "
                                          "alpha 2e-4, max_iter 10000, tol 1e-4",
            "ms": round(ms, 3), "n_iter": int(it), "nonzero": int((w != 0).sum().item()),
            "us_per_sweep": round(ms * 1e3 / max(it, 1), 2), "converged": bool(gap < tol_y)}


def bench_ingest(reps, A=10000, T=5040, K=3):
    import torch
    from afm import _lib
    from afm.grid import pack_bits
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    lda = (A + 63) // 64 * 64
    valid = torch.zeros((T, lda), dtype=torch.bool, device="cuda")
    valid[:, :A] = torch.rand((T, A), generator=g, device="cuda") < 0.95
    bits = pack_bits(valid)
    base = torch.randn((K, T, lda), generator=g, dtype=torch.float64, device="cuda")
    base[torch.rand((K, T, lda), generator=g, device="cuda") < 0.2] = float("nan")
    planes = base.clone()
    scratch = torch.empty_like(planes)
    n = int(valid.sum().item())
    x = torch.randn(n, generator=g, dtype=torch.float64, device="cuda") * 0.02
    cnt = valid.sum(dim=1).to(torch.int64)
    off = torch.zeros(T + 1, dtype=torch.int64, device="cuda")
    off[1:] = torch.cumsum(cnt, 0)
    out = torch.empty_like(x)
    xs = torch.empty_like(x)
    h = _lib.Context.get(0).bind_stream()
    L, P = _lib.lib(), _lib.ptr

    def fill():
        planes.copy_(base)
        _lib.check(L.afm_ffill_f64(h, K, T, lda, P(planes), P(bits)))
        _lib.check(L.afm_date_mean_fill_f64(h, K, T, A, lda, P(planes), P(bits), P(scratch)))
    ms_copy = timed(lambda: planes.copy_(base), reps)
    ms_fill = timed(fill, reps) - ms_copy
    ms_dm = timed(lambda: _lib.check(L.afm_group_demean_f64(h, T, P(off), int(cnt.max().item()),
                                                             P(x), P(out), P(xs))), reps)
    return {"stage": "ingest", "workload": f"{K} value columns on a {A} x {T} union grid "
                                           f"({n} rows), excess demean over {n} reference rows",
            "fill_ms": round(ms_fill, 3), "demean_ms": round(ms_dm, 3),
            "rows_per_s": round(n / ((ms_fill + ms_dm) * 1e-3), 1)}


def bench_talib(reps, A=10000, T=5040):
    import torch
    import afm
    from afm.synthetic import make_panel
    from afm.talib_factors import TALIB_COLS, talib_panel
    g = afm.PanelGrid.from_panel(make_panel(A, T, seed=2023))
    out = torch.empty((TALIB_COLS, T, g.lda), dtype=torch.float64, device="cuda")
    ms = timed(lambda: talib_panel(g, out), reps)
    n = g.n_asset_days()
    byts = (16 + 8 * TALIB_COLS) * n
    return {"stage": "talib", "workload": f"{A} assets x {T} days, {TALIB_COLS} TA-Lib columns",
            "ms": round(ms, 3), "asset_days_per_s": round(n / (ms * 1e-3), 1),
            "GBps": round(byts / (ms * 1e-3) / 1e9, 1)}


def bench_intraday(reps, A=3000, T=2 * 252 * 390):
    """Config D both ways: time slabs over all assets (the default build, state carried across
    slabs) and asset groups over the whole series."""
    import torch
    from afm.intraday import (factor_panel_groups, factor_panel_slabs, group_blocks,
                              make_panel_device, slab_bars)
    g = make_panel_device(A, T, seed=2023)
    bars = int(g.valid.sum().item())
    byts = 816 * bars
    step = slab_bars(g)
    slabs = []
    factor_panel_slabs(g, lambda t0, t1, o, nf: slabs.append((t0, t1)), step)   # warm-up
    ms_s = timed(lambda: factor_panel_slabs(g, lambda *x: None, step), max(1, reps // 3))
    bpg = group_blocks(g)
    groups = []
    factor_panel_groups(g, lambda a0, a1, o, nf: groups.append((a0, a1)), bpg)   # warm-up
    ms_g = timed(lambda: factor_panel_groups(g, lambda *x: None, bpg), max(1, reps // 3))
    return {"stage": "intraday", "workload": f"config D: {A} assets x {T} 1-minute bars "
                                             f"({bars} present asset-bars), 98 factors",
            "slabs": {"n": len(slabs), "bars_per_slab": step, "ms": round(ms_s, 1),
                      "asset_bars_per_s": round(bars / (ms_s * 1e-3), 1),
                      "GBps": round(byts / (ms_s * 1e-3) / 1e9, 1)},
            "groups": {"n": len(groups), "blocks_per_group": bpg, "ms": round(ms_g, 1),
                       "asset_bars_per_s": round(bars / (ms_g * 1e-3), 1),
                       "GBps": round(byts / (ms_g * 1e-3) / 1e9, 1)},
            "algorithmic_GB": round(byts / 1e9, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    for nm, fn in (("zscore", bench_zscore), ("bootstrap", bench_bootstrap),
                   ("lasso", bench_lasso), ("ingest", bench_ingest), ("talib", bench_talib),
                   ("intraday", bench_intraday)):
        if a.only and a.only != nm:
            continue
        t0 = time.perf_counter()
        r = fn(a.reps)
        r["wall_s"] = round(time.perf_counter() - t0, 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Headline benchmark: asset-days/s for factor build + cross-sectional regression + KKT weights
(BASELINE.json ``metric``), SURVEY.md §8(d).

Workload (N=1): BASELINE.json configs[2] -- 10,000 assets x 20 years (5,040 trading days) daily
synthetic panel (seeded generator, SURVEY.md §8(d): ragged listings, 0.2% holes, 90% tradable),
inputs resident in HBM before the timed region.  One step = afm.pipeline.Pipeline.step(), the
reference chain that feeds PortfolioManager: 98-column factor build (NT:1-93) -> train-window
per-security z-score of the 97 features (KKT:424-458, the reference's split dates) -> pooled
train+valid Gram of [1, z_1..z_97, target] on fp64 MFMA (z applied on the fly) -> Lasso(alpha=2e-4)
(KKT:605-607) -> test predictions (KKT:612) -> rolling-252-day covariance + exact min-variance
KKT weights for top/bottom-10 books on every test date + PnL/turnover scan (KKT:976-977); side
streams: AlphaSignalAnalyzer on the predictions (KKT:630-631) and the per-date FM30 OLS +
Fama-MacBeth (north-star extension).

Usage: python bench.py [--gpus N --steps K --warmup W].  N > 1 runs one rank per GPU: under
torch.distributed.run (WORLD_SIZE set; --gpus must equal it), or, started bare, bench.py starts
``python -m torch.distributed.run --nproc-per-node N ... bench.py`` itself as a CHILD process
before anything imports torch or touches the GPU, passes rank 0's line through and exits with
the child's code (self_launch below).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "alpha-multi-factor-models_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E (MI355X_MICROARCH.md chip table)
F64_MFMA_PEAK_TFS = 78.6       # MI355X fp64 matrix peak (spec)
FACTOR_BYTES_PER_AD = 816      # 4 x 8 B inputs read + 98 x 8 B outputs written
# the factor stage without the two label planes (they run on a side stream beside the factor
# kernel: afm/pipeline.py): close + volume read, 96 columns written
FACTOR_BYTES_NO_LABELS = 784


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# per-launch HBM bytes from the latest PMC passes (tools/prof_counters.sh -> tools/pmc_traffic.py;
# FETCH_SIZE x2 and KiB corrections of MI355X_MICROARCH.md applied there)
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r6z_pmc_traffic.json")
# config D (the time-slab factor build): HBM bytes of one whole pass, every slab launch of the
# factor / masks / label kernels (tools/gpu_pmc_config_d.sh -> tools/pmc_pass.py)
PMC_CONFIG_D = os.path.join(ROOT, "profiles", "r6_pmc_config_d.json")
ROOF_KERNELS = {"factors": ("factor_panel_kernel", "masks_kernel", "labels_kernel"),
                "factors_nolabels": ("factor_panel_kernel", "masks_kernel"),
                "xs_gram": ("zgram_kernel<7, 1, true>",)}


def pmc_traffic(stage: str, assets: int, days: int):
    """HBM bytes per launch of the stage's kernels, or None when no PMC pass of this workload
    is on file."""
    try:
        with open(PMC_TRAFFIC) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("workload") != [assets, days]:
        return None
    ks = d.get("kernels", {})
    if not all(k in ks for k in ROOF_KERNELS[stage]):
        return None
    return sum(ks[k]["hbm_bytes"] for k in ROOF_KERNELS[stage])


# SURVEY.md §8(d) conversion, measured in the build container on the same 500 x 2,520 panel
# (seed 2023): oracle/pandas_chain.py ran at 4,335 asset-days/s, the reference as written at
# 2,519 -- the restatement is 1.72x the reference's rate on identical input.
RESTATEMENT_OVER_REFERENCE = 4335.1 / 2519.0


def cpu_baseline(seed: int, assets: int = 500, days: int = 2520, max_dates: int = 40):
    """The reference's CPU path in its own call pattern (oracle/pandas_chain.py: per-security
    pandas factor loop, groupby z-score, scikit-learn Lasso, pandas analyzer, per-date all_df
    filter + SLSQP PortfolioManager loop), 1 core, at BASELINE config A (500 x 2,520, the
    reference's split rule).  Bounded sample: every stage runs in full except the per-date
    PortfolioManager loop, timed over its first ``max_dates`` rebalance dates and scaled to all
    of them (its cost is per date; the KKT:847 all_df filter inside it is O(panel) per date and
    is reported on its own, so the rate is given both as written and hot-path only).  The value
    path of a full run equals oracle/chain.py's bit for bit (tests/test_pandas_chain.py)."""
    from threadpoolctl import threadpool_limits

    from afm.synthetic import make_panel
    from oracle import pandas_chain
    p = make_panel(assets, days, seed=seed, tradable_p=0.9)
    n_ad = int(p.valid.sum())
    tm = {}
    with threadpool_limits(1):                                       # 1 core, BLAS included
        t0 = time.perf_counter()
        pandas_chain.run_chain(p, "2006-12-29", "2007-12-31", timings=tm, max_dates=max_dates)
        wall = time.perf_counter() - t0
    nd, nd_all = tm["dates"], tm["dates_total"]
    pre = sum(tm[k] for k in ("factors", "zscore", "lasso", "analyzer"))
    port = tm["portfolio"] / nd * nd_all                             # the whole loop
    filt = tm["filter_847"] / nd * nd_all
    total = pre + port
    value = n_ad / total
    return {"value": round(value, 1), "unit": "asset-days/s", "cores": 1, "kind": "port",
            "value_hot_path": round(n_ad / (total - filt), 1),
            "value_reference_equiv": round(value / RESTATEMENT_OVER_REFERENCE, 1),
            "filter_847_s": round(filt, 2),
            "sample": f"pandas/scikit-learn/SLSQP restatement of the reference call pattern "
                      f"(oracle/pandas_chain.py) at config A, {assets} assets x {days} days = "
                      f"{n_ad} asset-days: factors {tm['factors']:.2f}s, zscore "
                      f"{tm['zscore']:.2f}s, lasso {tm['lasso']:.2f}s, analyzer "
                      f"{tm['analyzer']:.2f}s run in full; the PortfolioManager loop timed on "
                      f"{nd} of {nd_all} rebalance dates ({tm['portfolio']:.2f}s, of which the "
                      f"KKT:847 all_df filter {tm['filter_847']:.2f}s) and scaled per date to "
                      f"{port:.1f}s (filter {filt:.1f}s); {wall:.1f}s wall.  value = as written; "
                      f"value_hot_path = without the KKT:847 filter; value_reference_equiv = "
                      f"value / {RESTATEMENT_OVER_REFERENCE:.2f}, the restatement/reference "
                      f"rate ratio measured in the build container on the same 500 x 2,520 "
                      f"panel (4,335 vs 2,519 asset-days/s, SURVEY.md §8(d))"}


def cpu_port(seed: int, assets: int = 150, days: int = 2520):
    """Secondary line: the vectorised oracle chain (oracle/chain.py: C factor restatement, numpy
    z-score, scikit-learn Lasso, exact-QP PortfolioManager, analyzer, per-date FM lstsq), 1 core."""
    from threadpoolctl import threadpool_limits

    from afm.pipeline import FM30
    from afm.synthetic import make_panel
    from oracle import chain
    p = make_panel(assets, days, seed=seed, tradable_p=0.9)
    n_ad = int(p.valid.sum())
    tm = {}
    with threadpool_limits(1):
        t0 = time.perf_counter()
        chain.run_chain(p, "2006-12-29", "2007-12-31", fm_features=FM30, timings=tm)
        total = time.perf_counter() - t0
    return {"value": round(n_ad / total, 1), "unit": "asset-days/s", "cores": 1, "kind": "port",
            "sample": f"oracle chain (oracle/chain.py) on {assets} assets x {days} days = {n_ad} "
                      f"asset-days: " + ", ".join(f"{k} {v:.2f}s" for k, v in tm.items())}


def kernel_times(evs: list) -> dict:
    """Mean device time (ms) of each KERNEL_MARKS pair the timed steps recorded (the one-pass
    factor call and the pooled Gram's partial kernel, on the main stream); marks a step path
    does not record (time slabs, the early z statistics) are left out."""
    from afm.pipeline import KERNEL_MARKS
    out = {}
    for k in KERNEL_MARKS:
        try:
            out[k] = sum(e[k][0].elapsed_time(e[k][1]) for e in evs) / len(evs)
        except (KeyError, RuntimeError, ValueError):   # a pair the path never recorded
            pass
    return out


def rooflines(pipe, stage_ms: dict, n_ad_local: int, world: int, assets: int, days: int,
              kms: dict | None = None):
    """The factor kernel (HBM) and pooled Gram (fp64 MFMA) roofline objects of one timed
    Pipeline, ranked by their stage's device time (dominant first).  ``achieved`` divides by the
    kernel's own event time when the step recorded it (``kernel_times``), else by its stage's."""
    kms = kms or {}
    labels_in = world == 1 and pipe.labels_in_factor_stage
    fac_bytes = FACTOR_BYTES_PER_AD if labels_in else FACTOR_BYTES_NO_LABELS
    fac_ms = kms.get("k_factor", stage_ms["factors"])
    gram_ms = kms.get("k_gram", stage_ms["xs_gram"])
    fac_gbs = fac_bytes * n_ad_local / (fac_ms * 1e-3) / 1e9
    p2 = pipe.p2
    rows_tv = float(pipe.pool_g[0, 0, 0].item())           # pooled rows (n of the Gram)
    if pipe.sp.dup:
        rows_tv -= float(pipe.te_gram[0, 0, 0].item())       # the duplicate is not recomputed
    rows_tv /= (world if world > 1 else 1)
    gram_tfs = rows_tv * p2 * (p2 + 1) / (gram_ms * 1e-3) / 1e12
    single = world == 1
    fac = {"bound": "hbm", "achieved": round(fac_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(fac_gbs / HBM_PEAK_GBS, 4),
           "traffic": None,
           "kernel": ("factor_panel_kernel + masks_kernel (one launch%s)" % (
               ", label planes inside" if labels_in else "; label planes on a side stream")
               if "k_factor" in kms else
               "factor_panel_kernel (+ masks, row-bit kernels%s)" % (
                   ", label planes" if labels_in else "; label planes on a side stream")),
           "kernel_ms": round(fac_ms, 3), "stage_ms": round(stage_ms["factors"], 3),
           "algorithmic_GB": round(fac_bytes * n_ad_local / 1e9, 3)}
    tb = (pmc_traffic("factors" if labels_in else "factors_nolabels", assets, days)
          if single else None)
    if tb is not None:
        fac["traffic"] = round(tb / 1e9, 3)
        fac["traffic_unit"] = "GB per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)"
    gram = {"bound": "mfma", "achieved": round(gram_tfs, 2), "peak": F64_MFMA_PEAK_TFS,
            "unit": "TFLOP/s", "frac": round(gram_tfs / F64_MFMA_PEAK_TFS, 4),
            "traffic": None,
            "kernel": ("zgram_kernel<7,1> (pooled train+valid Gram partials; the stage adds the "
                       "tree merges)" if "k_gram" in kms else
                       "zgram_kernel<7,1> + tree_merge_kernel (pooled train+valid Gram)"),
            "kernel_ms": round(gram_ms, 3), "stage_ms": round(stage_ms["xs_gram"], 3),
            "algorithmic_GFLOP": round(rows_tv * p2 * (p2 + 1) / 1e9, 3)}
    tg = pmc_traffic("xs_gram", assets, days) if single else None
    if tg is not None:
        gram["traffic"] = round(tg / 1e9, 3)
    ranked = sorted([(stage_ms["factors"], fac), (stage_ms["xs_gram"], gram)], key=lambda x: -x[0])
    return [r[1] for r in ranked]


def config_b_line(seed: int, steps: int, warmup: int) -> dict:
    """BASELINE configs[1]: 3,000 assets x 20 years daily (5,040 days) through the same step --
    factors -> z-score -> pooled Gram -> Lasso -> predict -> KKT rebalance -> PnL, with the
    per-date Fama-MacBeth regressions on FM30 (~30 factors) and the analyzer's IC series on the
    side streams, exactly the stages config B names."""
    import torch
    import afm
    from afm.pipeline import PipelineConfig
    from afm.synthetic import make_panel
    A, T = 3000, 5040
    grid = afm.PanelGrid.from_panel(make_panel(A, T, seed=seed, tradable_p=0.9))
    out = variant_line(grid, PipelineConfig(), steps, warmup,
                       f"config B (BASELINE configs[1]): {A} assets x {T} days, FM30 per-date "
                       f"Fama-MacBeth + IC series beside the headline chain", roof=(A, T))
    del grid
    torch.cuda.empty_cache()
    return out


def config_d_line(seed: int, reps: int) -> dict:
    """BASELINE configs[3]: 3,000 assets x 2 years of 1-minute bars (2 x 252 x 390 = 196,560
    bars, ~5.9e8 asset-bars), the 98-column factor build by time slabs over all assets
    (afm.intraday.factor_panel_slabs: every recurrence state and observation ring carried from
    slab to slab; the output planes of one slab at a time fit HBM)."""
    import torch
    from afm.intraday import factor_panel_slabs, make_panel_device, slab_bars
    A, T = 3000, 2 * 252 * 390
    g = make_panel_device(A, T, seed=seed)
    bars = int(g.valid.sum().item())
    step = slab_bars(g)
    n_slabs = factor_panel_slabs(g, lambda *x: None, step)           # warm-up pass
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        factor_panel_slabs(g, lambda *x: None, step)
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / reps
    byts = FACTOR_BYTES_PER_AD * bars
    gbs = byts / (ms * 1e-3) / 1e9
    traffic = None
    try:
        with open(PMC_CONFIG_D) as f:
            pd = json.load(f)
        if pd.get("workload") == [A, T]:
            traffic = round(pd["hbm_bytes_per_pass"] / 1e9, 1)
    except (OSError, ValueError, KeyError):
        pass
    del g
    torch.cuda.empty_cache()
    return {"what": f"config D (BASELINE configs[3]): {A} assets x {T} one-minute bars, 98 "
                    f"factors by time slab ({n_slabs} slabs of {step} bars, state carried)",
            "reps": reps, "ms_per_pass": round(ms, 2), "asset_bars": bars,
            "value": round(bars / (ms * 1e-3), 1), "unit": "asset-bars/s",
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "traffic_unit": "GB per pass (PMC FETCH_SIZE x2 + WRITE_SIZE, every "
                                         "slab launch)",
                         "kernel": "factor_panel_kernel (+ masks, label planes) per slab",
                         "algorithmic_GB": round(byts / 1e9, 1),
                         "bytes_per_unit": FACTOR_BYTES_PER_AD}}


def config_e_line(seed: int, reps: int, n_paths: int = 1024) -> dict:
    """BASELINE configs[4]: bootstrap backtest -- 1,024 resampled date paths x 5,000 assets.  The
    panel's step supplies the Lasso predictions; timed: the batched KKT rebalance of every test
    date once (books, rolling-252 pairwise covariance, exact box-QP weights; path-independent)
    + the 1,024 paths' turnover alignment and value recursion (KKT:842-892 per path step)."""
    import torch
    import afm
    from afm.pipeline import Pipeline, PipelineConfig
    from afm.portfolio import bootstrap_paths, bootstrap_pnl, rebalance
    from afm.synthetic import make_panel
    A, T = 5000, 5040
    grid = afm.PanelGrid.from_panel(make_panel(A, T, seed=seed, tradable_p=0.9))
    cfg = PipelineConfig()
    pipe = Pipeline(grid, cfg)
    pipe.step()
    torch.cuda.synchronize()
    paths = torch.from_numpy(bootstrap_paths(pipe.nd, n_paths, seed=2023)).cuda()
    steps = int(paths.shape[1])
    res = {}

    def reb():
        res["reb"] = rebalance(pipe.pred, grid.tbits, pipe.target, pipe.zrows_full, grid.close,
                               pipe.tmr, pipe.rdates, A=A, top_n=cfg.top_n, window=cfg.window,
                               h_range=(0, pipe.sp.tr1), lo=cfg.lo, hi=cfg.hi)

    def boot():
        res["boot"] = bootstrap_pnl(res["reb"], pipe.pred, pipe.rdates, paths, rate=cfg.rate)
    reb()
    boot()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    t_reb = t_boot = 0.0
    for _ in range(reps):
        ev[0].record()
        reb()
        ev[1].record()
        boot()
        ev[2].record()
        torch.cuda.synchronize()
        t_reb += ev[0].elapsed_time(ev[1])
        t_boot += ev[1].elapsed_time(ev[2])
    t_reb /= reps
    t_boot /= reps
    ok = bool(torch.isfinite(res["boot"]["value"]).all().item())
    n_ps = n_paths * steps
    # the per-path-step O(A) work is the id-union alignment (KKT:839): both slots' prediction
    # presence words read (2 x lda / 8 B), plus the step's 4 PnL sums read and 4 series written
    byts = n_ps * (2 * grid.lda // 8 + 4 * 8 + 4 * 8)
    gbs = byts / (t_boot * 1e-3) / 1e9
    nd = pipe.nd
    del pipe, res
    torch.cuda.empty_cache()
    return {"what": f"config E (BASELINE configs[4]): {n_paths} bootstrap paths x {steps} "
                    f"rebalance dates, {A} assets: batched KKT rebalance of the {nd} dates + the "
                    f"paths' turnover alignment and value recursion",
            "reps": reps, "rebalance_ms": round(t_reb, 3), "paths_ms": round(t_boot, 3),
            "ms_per_pass": round(t_reb + t_boot, 3), "path_steps": n_ps,
            "value": round(n_ps / ((t_reb + t_boot) * 1e-3), 1), "unit": "path-steps/s",
            "asset_path_steps_per_s": round(A * n_ps / ((t_reb + t_boot) * 1e-3), 1),
            "all_paths_finite": ok,
            "roofline": {"bound": "hbm", "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 6), "traffic": None,
                         "kernel": "afm_bootstrap_pnl_f64 (pred_bits + pair_union + "
                                   "turnover_terms + pnl_scan kernels); latency-bound: one "
                                   "sequential value recursion per path",
                         "kernel_ms": round(t_boot, 3), "algorithmic_GB": round(byts / 1e9, 3)}}


def variant_line(grid, cfg, steps: int, warmup: int, what: str, roof=None) -> dict:
    """Secondary timed line on the same resident panel: a PipelineConfig variant of the headline
    step, W untimed + K timed steps bracketed by synchronize, per-stage device times."""
    import numpy as np
    import torch
    from afm.pipeline import KERNEL_MARKS, PIPELINE_STAGES, Pipeline
    pipe = Pipeline(grid, cfg)
    for _ in range(warmup):
        pipe.step()
    evs = [{st: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            for st in PIPELINE_STAGES + KERNEL_MARKS} for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        pipe.step(evs[k])
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    stage_ms = {st: round(sum(e[st][0].elapsed_time(e[st][1]) for e in evs) / steps, 3)
                for st in PIPELINE_STAGES}
    s = pipe.summary()
    st = np.bincount(s["status"], minlength=3)
    out = {"what": what, "steps": steps, "warmup": warmup, "ms_per_step": round(ms, 3),
           "value": round(grid.n_asset_days() / (ms * 1e-3), 1), "unit": "asset-days/s",
           "stage_ms": stage_ms, "top_n": cfg.top_n, "features": pipe.p,
           "lasso_nnz": s["lasso_nnz"], "lasso_n_iter": s["lasso_n_iter"],
           "qp_status_counts": st.tolist(), "final_value": s["final_value"]}
    w = pipe.reb["weights"][:, :, :cfg.top_n].cpu().numpy()
    out["weights_at_bounds_frac"] = round(float(((w <= cfg.lo) | (w >= cfg.hi)).mean()), 4)
    if roof is not None:
        out["assets"], out["days"] = roof
        rl = rooflines(pipe, stage_ms, grid.n_asset_days(), 1, *roof, kms=kernel_times(evs))
        out["roofline"], out["roofline_next"] = rl[0], rl[1]
        out["fm_ms"] = stage_ms["fm"]
        out["ic_mean"] = [round(float(x), 6) for x in s.get("ic_mean", [])]
    del pipe
    torch.cuda.empty_cache()
    return out


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(gpus: int, argv: list) -> int:
    """``bench.py --gpus N`` (N > 1) started without a launcher: run the same command line under
    ``torch.distributed.run`` (one rank per GPU, rendezvous on 127.0.0.1) as a child process --
    never exec: this process has not imported torch nor touched the GPU, and it stays the parent.
    Rank 0's JSON line is passed through on stdout; everything else the job prints goes to
    stderr.  Returns the child's exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    log(f"[bench] --gpus {gpus}: launching {gpus} ranks: {' '.join(cmd)}")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1)
    assert proc.stdout is not None
    for line in proc.stdout:
        s = line.strip()
        if s.startswith("{") and s.endswith("}"):
            print(s, flush=True)
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    return proc.wait()


def launch_world(gpus) -> tuple:
    """(world, must_self_launch) from --gpus and the launcher's WORLD_SIZE.  Under a launcher,
    --gpus (when given) must equal WORLD_SIZE."""
    env = os.environ.get("WORLD_SIZE")
    if env is not None:
        world = int(env)
        if gpus is not None and gpus != world:
            raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE="
                             f"{world} ranks")
        return world, False
    n = 1 if gpus is None else gpus
    if n < 1:
        raise SystemExit(f"bench.py: --gpus {n}")
    return n, n > 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default 1, or WORLD_SIZE under a launcher); N > 1 "
                         "without a launcher starts torch.distributed.run as a child process")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--assets", type=int, default=10000)
    ap.add_argument("--days", type=int, default=5040)
    ap.add_argument("--seed", type=int, default=2023)
    ap.add_argument("--top-n", type=int, default=10)
    ap.add_argument("--train-end", default=None, help="PipelineConfig.train_end (small panels)")
    ap.add_argument("--valid-end", default=None, help="PipelineConfig.valid_end (small panels)")
    ap.add_argument("--window", type=int, default=None,
                    help="PipelineConfig.window (rolling covariance days)")
    ap.add_argument("--fm-free-cus", type=int, default=None,
                    help="PipelineConfig.fm_free_cus (CUs the FM side stream leaves free)")
    ap.add_argument("--fm-fork", default=None,
                    help="PipelineConfig.fm_fork (where the FM Grams fork off the main stream)")
    ap.add_argument("--fm-grid", type=int, default=None,
                    help="PipelineConfig.fm_grid (A/B; default: one FM workgroup per CU)")
    ap.add_argument("--zstats-slabs", type=int, default=None,
                    help="PipelineConfig.zstats_slabs (A/B; default: the pipeline's auto rule)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="time what ONE rank of an N-GPU job computes, on one GPU (collectives "
                         "replaced by local copies, afm.sharded.EmulatedComm): a per-rank proxy, "
                         "not a result of the job")
    ap.add_argument("--early-fwd", type=int, default=None,
                    help="PipelineConfig.early_fwd 0/1 (A/B; default: on)")
    ap.add_argument("--reb-split", type=int, default=None,
                    help="PipelineConfig.reb_split (N > 1: 1 = rebalance dates split over the "
                         "ranks + all-gather, 0 = every rank all dates)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the config B / D / E lines (N = 1 only)")
    ap.add_argument("--config-only", choices=("b", "d", "e"), default=None,
                    help="run only that config line and print it (profiling runs)")
    ap.add_argument("--no-variants", action="store_true",
                    help="skip the top_n_100 / dense_lasso secondary lines (N = 1 only)")
    args = ap.parse_args()
    world, spawn = launch_world(args.gpus)
    if spawn and not args.config_only:
        if args.emulate_world:
            raise SystemExit("bench.py: --emulate-world is a one-GPU proxy; drop --gpus")
        sys.exit(self_launch(world, sys.argv[1:]))

    import numpy as np
    import torch
    import torch.distributed as dist

    import afm
    from afm.pipeline import PIPELINE_STAGES, Pipeline, PipelineConfig
    from afm.synthetic import make_panel

    if args.config_only:
        fn = {"b": lambda: config_b_line(args.seed, max(2, min(args.steps, 5)), 1),
              "d": lambda: config_d_line(args.seed, 2),
              "e": lambda: config_e_line(args.seed, 3)}[args.config_only]
        print(json.dumps({"config_" + args.config_only: fn()}), flush=True)
        return

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("AFM_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "gloo" and ndev:
        local = local % ndev          # rehearsal only: gloo ranks may share a GPU
    elif ndev and local >= ndev:
        raise SystemExit(f"LOCAL_RANK {local} but only {ndev} visible GPUs")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)

    t0 = time.perf_counter()
    p = make_panel(args.assets, args.days, seed=args.seed, tradable_p=0.9)
    grid = afm.PanelGrid.from_panel(p, device=dev)
    del p
    n_ad = grid.n_asset_days()                         # the whole panel (strong scaling)
    place = {}
    if args.fm_free_cus is not None:
        place["fm_free_cus"] = args.fm_free_cus
    if args.fm_fork is not None:
        place["fm_fork"] = args.fm_fork
    if args.zstats_slabs is not None:
        place["zstats_slabs"] = args.zstats_slabs
    if args.fm_grid is not None:
        place["fm_grid"] = args.fm_grid
    if args.reb_split is not None:
        place["reb_split"] = bool(args.reb_split)
    if args.early_fwd is not None:
        place["early_fwd"] = bool(args.early_fwd)
    for k in ("train_end", "valid_end", "window"):
        if getattr(args, k) is not None:
            place[k] = getattr(args, k)
    cfg = PipelineConfig(top_n=args.top_n, **place)
    if world > 1:
        from afm.sharded import EXCHANGE_STAGES, Comm, ShardedPipeline
        pipe = ShardedPipeline(grid, Comm(), cfg)
        stages = EXCHANGE_STAGES
        n_ad_local = pipe.n_asset_days_local()
    elif args.emulate_world > 1:
        from afm.sharded import EXCHANGE_STAGES, EmulatedComm
        pipe = Pipeline(grid, cfg, EmulatedComm(args.emulate_world, 0))
        stages = EXCHANGE_STAGES
        n_ad_local = pipe.n_asset_days_local()
    else:
        pipe = Pipeline(grid, cfg)
        stages = PIPELINE_STAGES
        n_ad_local = n_ad
    torch.cuda.synchronize()
    log(f"[rank {rank}] panel {grid.A}x{grid.T} ({n_ad} asset-days, {n_ad_local} in this rank's "
        f"factor shard) ready in {time.perf_counter() - t0:.1f}s; split {pipe.sp}")

    for _ in range(args.warmup):
        pipe.step()
    torch.cuda.synchronize()
    if rank == 0 and args.warmup:
        s = pipe.summary()
        log(f"[rank 0] warmup: final value {s['final_value']:.9g}, sharpe {s['sharpe']:.6g}, "
            f"lasso n_iter {s['lasso_n_iter']} nnz {s['lasso_nnz']}, FM rank counts "
            f"{np.bincount(s['fm_rank'])[-2:]}, k {np.bincount(s['k'])[-2:]}, qp status "
            f"{np.bincount(s['status'])}, mean IC {s.get('ic_mean')}")

    from afm.pipeline import KERNEL_MARKS
    evs = [{st: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            for st in stages + KERNEL_MARKS} for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        pipe.step(evs[k])
    issued = time.perf_counter() - t0          # host time to enqueue the K steps
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stage_ms = {st: sum(e[st][0].elapsed_time(e[st][1]) for e in evs) / args.steps
                for st in stages}

    total_ad = n_ad
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device="cpu" if backend == "gloo" else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])

    if args.emulate_world > 1:          # per-rank proxy: no headline line
        ms = elapsed / args.steps * 1e3
        print(json.dumps({"emulated_world": args.emulate_world, "rank": 0,
                          "assets_local": pipe.A_r, "ms_per_step": round(ms, 3),
                          "host_issue_ms_per_step": round(issued / args.steps * 1e3, 3),
                          "stage_ms": {k: round(v, 3) for k, v in stage_ms.items()},
                          "note": "one rank's kernels on one GPU, collectives replaced by local "
                                  "copies (afm.sharded.EmulatedComm); no communication time"}),
              flush=True)
        return
    final_value = pipe.summary()["final_value"] if rank == 0 else None
    if rank == 0:
        ms = elapsed / args.steps * 1e3
        # roofline of the two dominant kernels, ranked by per-step device time: the factor panel
        # (HBM: 816 B per asset-day; 784 B without the two label planes, which
        # run on a side stream beside the factor kernel) and the pooled Gram (fp64 MFMA:
        # rows * (p+2)(p+3) flops over the train + valid rows, zpool + tree merges).
        ranked = rooflines(pipe, stage_ms, n_ad_local, world, args.assets, args.days,
                           kernel_times(evs))
        res = {
            "metric": "asset-days/sec, factor build+XS regression+KKT (10k assets x 20y), "
                      "1/2/4/8 GPU",
            "value": round(total_ad / (ms * 1e-3), 1),
            "unit": "asset-days/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            # host time to enqueue one step (rank 0): below ms_per_step the GPU sets the pace
            "host_issue_ms_per_step": round(issued / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic (seeded OHLCV panel, SURVEY.md §8(d))",
            "config": {"workload": f"{args.assets} assets x {args.days} days daily panel: 98 "
                                   f"factors -> train-window z-score (97 features) -> per-date "
                                   f"MFMA Grams -> pooled Lasso -> predict -> rolling-252 cov + "
                                   f"exact KKT top/bottom-{args.top_n} -> PnL; side: analyzer "
                                   f"(IC/layers/top-10) + per-date FM30 OLS",
                       "assets": args.assets, "days": args.days, "asset_days": total_ad,
                       "split": {"train_end": cfg.train_end, "valid_end": cfg.valid_end},
                       "parallelism": (f"asset shards (factors, block Grams) + date shards "
                                       f"(solves, rebalance) x{world}") if world > 1
                       else "single"},
            "stage_ms": {k: round(v, 3) for k, v in stage_ms.items()},
            "roofline": ranked[0],
            "roofline_next": ranked[1],
            # the portfolio's last value after the timed steps (KKT:892): the same for every N
            "final_value": final_value,
        }
        if world == 1 and not args.no_variants:
            # secondary lines the headline step never exercises: the active-set KKT QP on
            # 100-name books (SURVEY §8(d) config C stress), and a dense Lasso / predict (a
            # stated non-reference design: the 96 factors without tmr_ret1d, KKT:433-443)
            from dataclasses import replace

            from afm.pipeline import DENSE_ALPHA, DENSE_FEATURES
            del pipe
            torch.cuda.empty_cache()
            vs, vw = max(2, min(args.steps, 5)), 1
            res["top_n_100"] = variant_line(grid, replace(cfg, top_n=100), vs, vw,
                                            "headline step with top_n = 100 (KKT:796 stress)")
            res["dense_lasso"] = variant_line(
                grid, replace(cfg, features=DENSE_FEATURES, alpha=DENSE_ALPHA), vs, vw,
                f"variant of KKT:433-443 / KKT:605: features without tmr_ret1d (96 columns), "
                f"Lasso alpha {DENSE_ALPHA:g} -- a dense fit, so the predict reads its support")
        if world == 1 and not args.no_configs:
            # the other BASELINE configs' throughput (north_star: "throughput across the
            # configs"), each on its own resident synthetic panel
            cs, cw = max(2, min(args.steps, 5)), 1
            res["config_b"] = config_b_line(args.seed, cs, cw)
            res["config_d"] = config_d_line(args.seed, 2)
            res["config_e"] = config_e_line(args.seed, 3)
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.seed)
            res["cpu_baseline_port"] = cpu_port(args.seed)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

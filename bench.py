#!/usr/bin/env python3
"""Headline benchmark: asset-days/s for factor build + cross-sectional regression + KKT weights
(BASELINE.json ``metric``), SURVEY.md §8(d).

Workload (N=1): BASELINE.json configs[2] -- 10,000 assets x 20 years (5,040 trading days) daily
synthetic panel (seeded generator, SURVEY.md §8(d): ragged listings, 0.2% holes), inputs
resident in HBM before the timed region.  One step = afm.pipeline.Pipeline.step(): 98-column
factor build, per-date OLS of next-day excess return on all 96 factors (fp64 MFMA Grams) + FM
stats, pooled OLS over the train+valid dates, predictions on the test dates (last 20%),
rolling-252-day covariance + exact min-variance KKT weights for top/bottom-10 books on every
test date, PnL/turnover scan.

Usage: python bench.py [--gpus N --steps K --warmup W]; N>1 is launched by torch.distributed.run
(one rank per GPU).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "alpha-multi-factor-models_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E (MI355X_MICROARCH.md chip table)
F64_MFMA_PEAK_TFS = 78.6       # MI355X fp64 matrix peak (spec)
FACTOR_BYTES_PER_AD = 816      # 4 x 8 B inputs read + 98 x 8 B outputs written


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# per-launch HBM bytes from the latest PMC passes (tools/prof_counters.sh -> tools/pmc_traffic.py;
# FETCH_SIZE x2 and KiB corrections of MI355X_MICROARCH.md applied there)
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "pmc_traffic.json")
ROOF_KERNELS = {"factors": ("factor_panel_kernel", "masks_kernel", "labels_kernel"),
                "xs_gram": ("gram_kernel",)}


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


def cpu_baseline(seed: int, assets: int = 500, days: int = 2520):
    """The oracle chain (C factor restatement + numpy per-date lstsq + sklearn pooled OLS +
    numpy/Python portfolio with the exact QP), 1 core, on config A (500 assets x 2520 days)."""
    import numpy as np
    from threadpoolctl import threadpool_limits

    import oracle
    from oracle import pipeline as PL
    from oracle import portfolio as PF
    from afm.synthetic import make_panel
    p = make_panel(assets, days, seed=seed)
    v = p.valid[:, :p.A]
    aa, tt = np.nonzero(v.T)
    off = np.r_[0, np.cumsum(v.sum(axis=0))].astype(np.int64)
    cols = [np.ascontiguousarray(x[tt, aa]) for x in (p.close, p.volume, p.ret1d, p.excess)]
    n_ad = len(tt)
    limiter = threadpool_limits(1)                                       # 1 core, BLAS included
    t0 = time.perf_counter()
    fac = oracle.factors_long(off, *cols)                               # factors
    t1 = time.perf_counter()
    X, y = fac[:, :96], fac[:, 96]
    use = np.isfinite(X).all(axis=1) & np.isfinite(y)
    T = days
    t_test = int(T * 0.8)
    PL.xs_ols(tt[use], X[use], y[use])                                   # per-date OLS
    t2 = time.perf_counter()
    tv = use & (tt < t_test)
    b0, b = PL.pooled_ols(X[tv], y[tv])                                  # pooled OLS
    te = use & (tt >= t_test) & (tt < T - 1)
    pred = b0 + X[te] @ b
    t3 = time.perf_counter()
    ids = p.ids[aa]
    dates = p.dates[tt].astype(np.int64)
    trad = p.tradable[tt, aa]
    PF.run_portfolio(dates[te], ids[te], pred, dates, ids, y, dates, ids, trad,   # KKT stage
                     cols[0], fac[:, 97], window=252)
    t4 = time.perf_counter()
    limiter.unregister() if hasattr(limiter, "unregister") else None
    total = t4 - t0
    return {"value": round(n_ad / total, 1), "unit": "asset-days/s", "cores": 1, "kind": "port",
            "sample": f"oracle chain on config A ({assets} assets x {days} days = {n_ad} "
                      f"asset-days): factors {t1 - t0:.2f}s, per-date OLS {t2 - t1:.2f}s, pooled "
                      f"OLS+predict {t3 - t2:.2f}s, rebalance+KKT+PnL {t4 - t3:.2f}s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--assets", type=int, default=10000)
    ap.add_argument("--days", type=int, default=5040)
    ap.add_argument("--seed", type=int, default=2023)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    import afm
    from afm.pipeline import PIPELINE_STAGES, Pipeline
    from afm.synthetic import make_panel

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the multi-rank path on a box with fewer GPUs than ranks: ranks share devices
    # round-robin and AFM_BENCH_BACKEND=gloo replaces RCCL (the driver's N-GPU runs use neither)
    ndev = torch.cuda.device_count()
    if ndev:
        local = local % ndev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("AFM_BENCH_BACKEND", "nccl")
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)

    t0 = time.perf_counter()
    p = make_panel(args.assets, args.days, seed=args.seed)
    grid = afm.PanelGrid.from_panel(p, device=dev)
    del p
    n_ad = grid.n_asset_days()                         # the whole panel (strong scaling)
    if world > 1:
        from afm.sharded import EXCHANGE_STAGES, Comm, ShardedPipeline
        pipe = ShardedPipeline(grid, Comm())
        stages = EXCHANGE_STAGES
        n_ad_local = pipe.n_asset_days_local()
    else:
        pipe = Pipeline(grid)
        stages = PIPELINE_STAGES
        n_ad_local = n_ad
    torch.cuda.synchronize()
    log(f"[rank {rank}] panel {grid.A}x{grid.T} ({n_ad} asset-days, {n_ad_local} in this rank's "
        f"factor shard) ready in {time.perf_counter() - t0:.1f}s")

    for _ in range(args.warmup):
        pipe.step()
    torch.cuda.synchronize()
    if rank == 0 and args.warmup:
        s = pipe.summary()
        log(f"[rank 0] warmup: final value {s['final_value']:.6g}, sharpe {s['sharpe']:.4g}, "
            f"per-date ranks {np.bincount(s['ranks'])[-3:]}, qp status {np.bincount(s['status'])}")

    evs = [{st: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            for st in stages} for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        pipe.step(evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stage_ms = {st: sum(e[st][0].elapsed_time(e[st][1]) for e in evs) / args.steps
                for st in stages}

    total_ad = n_ad
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])

    if rank == 0:
        ms = elapsed / args.steps * 1e3
        # roofline of the dominant kernel: factor panel (HBM) or the per-date Gram (fp64 MFMA)
        p = pipe.p
        fac_gbs = FACTOR_BYTES_PER_AD * n_ad_local / (stage_ms["factors"] * 1e-3) / 1e9
        if world == 1:      # stage xs_gram = the train+valid dates (the test dates: side stream)
            gram_rows = float(pipe.nobs[:pipe.t_test].sum().item())
        else:
            gram_rows = float(pipe.nobs.sum().item()) / world  # this rank's share of the rows
        gram_tfs = gram_rows * (p + 2) * (p + 3) / (stage_ms["xs_gram"] * 1e-3) / 1e12
        single = world == 1
        if stage_ms["factors"] >= stage_ms["xs_gram"]:
            tb = pmc_traffic("factors", args.assets, args.days) if single else None
            roof = {"bound": "hbm", "achieved": round(fac_gbs, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(fac_gbs / HBM_PEAK_GBS, 4),
                    "traffic": None if tb is None else round(tb / 1e9, 3),
                    "traffic_unit": "GB per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                    "algorithmic": round(FACTOR_BYTES_PER_AD * n_ad_local / 1e9, 3),
                    "kernel": "+".join(ROOF_KERNELS["factors"]),
                    "kernel_ms": round(stage_ms["factors"], 3)}
        else:
            tb = pmc_traffic("xs_gram", args.assets, args.days) if single else None
            roof = {"bound": "mfma", "achieved": round(gram_tfs, 2), "peak": F64_MFMA_PEAK_TFS,
                    "unit": "TFLOP/s", "frac": round(gram_tfs / F64_MFMA_PEAK_TFS, 4),
                    "traffic": None if tb is None else round(tb / 1e9, 3),
                    "traffic_unit": "GB per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                    "kernel": "gram_kernel", "kernel_ms": round(stage_ms["xs_gram"], 3)}
        res = {
            "metric": "asset-days/sec, factor build+XS regression+KKT (10k assets x 20y), "
                      "1/2/4/8 GPU",
            "value": round(total_ad / (ms * 1e-3), 1),
            "unit": "asset-days/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic (seeded OHLCV panel, SURVEY.md §8(d))",
            "config": {"workload": f"{args.assets} assets x {args.days} days daily panel: 98 "
                                   f"factors -> per-date OLS on 96 factors + FM -> pooled OLS -> "
                                   f"predict -> rolling-252 cov + exact KKT top/bottom-10 -> PnL",
                       "assets": args.assets, "days": args.days, "asset_days": total_ad,
                       "parallelism": (f"asset shards (factors, partial Grams) + date shards "
                                       f"(solves, rebalance) x{world}") if world > 1
                       else "single"},
            "stage_ms": {k: round(v, 3) for k, v in stage_ms.items()},
            "roofline": roof,
            "secondary": {"factor_panel_GBps": round(fac_gbs, 1),
                          "gram_TFLOPs": round(gram_tfs, 2)},
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.seed)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

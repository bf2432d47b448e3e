#!/usr/bin/env python3
"""Headline benchmark: asset-days/s for the factor-research hot path (BASELINE.json ``metric``).

Workload (N=1): BASELINE.json configs[2] -- 10,000 assets x 20 years (5,040 trading days) daily
synthetic panel (seeded generator of SURVEY.md §8(d), ragged listings, 0.2% holes), inputs
resident in HBM before the timed region.  One step = one pass of the hot path over the panel.

Usage: python bench.py [--gpus N --steps K --warmup W]; for N>1 the driver launches it with
torch.distributed.run (one rank per GPU).  Rank 0 prints ONE JSON line.
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

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
FACTOR_BYTES_PER_AD = 816      # 4 x 8 B inputs read + 98 x 8 B outputs written


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(seed: int):
    """The oracle (C restatement of No-talib.py, 1 thread) on a bounded sample: config A
    (500 assets x 2,520 days)."""
    import numpy as np

    import oracle
    from afm.synthetic import make_panel
    p = make_panel(500, 2520, seed=seed)
    v = p.valid[:, :p.A]
    aa, tt = np.nonzero(v.T)
    off = np.r_[0, np.cumsum(v.sum(axis=0))].astype(np.int64)
    cols = [np.ascontiguousarray(x[tt, aa]) for x in (p.close, p.volume, p.ret1d, p.excess)]
    oracle.factors_long(off[:3], *[c[: off[2]] for c in cols])      # warm the library
    t0 = time.perf_counter()
    reps = 0
    while True:
        oracle.factors_long(off, *cols)
        reps += 1
        if time.perf_counter() - t0 > 10.0 or reps >= 20:
            break
    dt = (time.perf_counter() - t0) / reps
    return {"value": round(len(tt) / dt, 1), "unit": "asset-days/s", "cores": 1, "kind": "port",
            "sample": f"factor build (oracle/factors_oracle.c, No-talib.py restated) on config A "
                      f"500 assets x 2520 days = {len(tt)} asset-days, {reps} reps"}


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
    from afm.synthetic import make_panel

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    # ---- synthetic panel (identical on every rank), asset shard of this rank -------------------
    t0 = time.perf_counter()
    p = make_panel(args.assets, args.days, seed=args.seed)
    lo = (args.assets * rank) // world
    hi = (args.assets * (rank + 1)) // world
    if world > 1:
        from afm.synthetic import Panel, round_up
        lda = round_up(hi - lo)

        def sl(x, fill):
            o = np.full((p.T, lda), fill, dtype=x.dtype)
            o[:, : hi - lo] = x[:, lo:hi]
            return o
        p = Panel(dates=p.dates, ids=p.ids[lo:hi], close=sl(p.close, np.nan),
                  volume=sl(p.volume, np.nan), ret1d=sl(p.ret1d, np.nan),
                  excess=sl(p.excess, np.nan), valid=sl(p.valid, False),
                  tradable=sl(p.tradable, False), group_id=p.group_id[lo:hi])
    grid = afm.PanelGrid.from_panel(p, device=dev)
    del p
    n_ad = grid.n_asset_days()
    out = torch.empty((afm.factors.N_FACTORS, grid.T, grid.lda), dtype=torch.float64, device=dev)
    nanfree = torch.zeros(((grid.T + 63) // 64, grid.lda), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    log(f"[rank {rank}] panel {grid.A}x{grid.T} ({n_ad} asset-days) ready in "
        f"{time.perf_counter() - t0:.1f}s")

    def step(ev=None):
        if ev is not None:
            ev[0].record()
        afm.factor_panel(grid, out, nanfree)
        if ev is not None:
            ev[1].record()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    fac_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps

    total_ad = n_ad
    if world > 1:
        t = torch.tensor([elapsed, float(n_ad)], dtype=torch.float64, device=dev)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed = float(mx[0])
        total_ad = int(sm[1])

    if rank == 0:
        ms = elapsed / args.steps * 1e3
        achieved = FACTOR_BYTES_PER_AD * n_ad / (fac_ms * 1e-3) / 1e9
        res = {
            "metric": "asset-days/sec, factor build+XS regression+KKT (10k assets x 20y), "
                      "1/2/4/8 GPU",
            "value": round(total_ad / (ms * 1e-3), 1),
            "unit": "asset-days/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic (seeded OHLCV panel, SURVEY.md §8(d))",
            "config": {"workload": f"factor build (98 cols, No-talib.py) on {args.assets} assets x "
                                   f"{args.days} days; stages: factors",
                       "assets": args.assets, "days": args.days, "asset_days": total_ad,
                       "parallelism": f"asset-shard x{world}" if world > 1 else "single"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None, "kernel": "factor_panel_kernel+labels_kernel",
                         "kernel_ms": round(fac_ms, 3)},
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.seed)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

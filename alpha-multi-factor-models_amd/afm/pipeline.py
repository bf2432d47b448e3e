"""The end-to-end hot path on one device: factor build -> cross-sectional regression -> KKT
weights -> PnL (BASELINE.json ``metric``).

One ``step()`` over a device-resident calendar-grid panel:

1. factors       afm_factors_f64: 98 planes + dropna / finite row masks
2. xs gram       afm_xs_gram_f64: per-date Gram of [1, 96 factors, target] on fp64 MFMA
3. xs solve      afm_ols_solve_f64 + afm_fama_macbeth_f64: per-date betas, FM mean / t
4. pooled OLS    afm_pool_moments_f64 + solve over the train+valid dates (the reference's
                 LinearRegression, KKT:582-583)
5. predict       afm_predict_f64 on the test dates
6. rebalance     afm_rebalance_f64: per test date top/bottom-n selection, rolling-window
                 pairwise covariance, exact box-QP weights (KKT:842-892)
7. pnl           afm_pnl_scan_f64: value / turnover recursion

All buffers are allocated once and there is no host synchronisation inside a step.  Stages
4-7 need only the Grams of the train+valid dates, and nothing downstream reads stage 3.  So the
main stream runs 1 -> 2 (train+valid dates) -> 4 -> 7 while a side stream, forked after the
pooled solve and joined at the end of the step, runs the test dates' Grams and stage 3.  The side
work fills the GPU while the main chain runs its latency-bound tail (the PnL scan uses one CU).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import _lib
from .factors import N_FACTORS, TARGET, TMR
from .grid import PanelGrid
from .portfolio import MAX_BOOK

STAGES = ("factors", "xs_gram", "xs_solve", "pooled_ols", "predict", "rebalance", "pnl")
# single-device step: xs_gram covers the train+valid dates (what the pooled OLS needs), the test
# dates' Grams (xs_gram_test) run on the side stream ahead of the per-date solve
PIPELINE_STAGES = STAGES + ("xs_gram_test",)


@dataclass
class PipelineConfig:
    cols: list = field(default_factory=lambda: list(range(96)))   # regressors: all 96 factors
    ycol: int = TARGET                                             # next-day excess return
    train_frac: float = 0.6        # dates [0, train) train, [train, test) valid, [test, T) test
    valid_frac: float = 0.2
    top_n: int = 10                # KKT:796
    window: int = 252              # rolling covariance window (north star); None = whole history
    lo: float = 0.0                # KKT:828
    hi: float = 0.1
    rate: float = 1e-4             # KKT:796
    tol: float = 1e-10


class Pipeline:
    def __init__(self, grid: PanelGrid, cfg: PipelineConfig | None = None):
        import torch
        self.g = grid
        self.cfg = cfg or PipelineConfig()
        dev = grid.device
        T, lda = grid.T, grid.lda
        nch = (T + 63) // 64
        self.T, self.lda, self.p = T, lda, len(self.cfg.cols)
        self.t_valid = int(T * self.cfg.train_frac)
        self.t_test = int(T * (self.cfg.train_frac + self.cfg.valid_frac))
        p2 = self.p + 2
        f64 = dict(dtype=torch.float64, device=dev)
        i64 = dict(dtype=torch.int64, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        self.out = torch.empty((N_FACTORS, T, lda), **f64)
        self.nanfree = torch.zeros((nch, lda), **i64)
        self.finite = torch.zeros((nch, lda), **i64)
        self.rows = torch.zeros((nch, lda), **i64)     # finite rows with a label (Gram rows)
        self.cols = torch.as_tensor(np.asarray(self.cfg.cols, dtype=np.int32), device=dev)
        self.gram = torch.empty((T, p2, p2), **f64)
        self.shift = torch.empty((T, p2), **f64)
        self.beta = torch.empty((T, self.p + 1), **f64)
        self.nobs = torch.empty(T, **f64)
        self.rank = torch.empty(T, **i32)
        self.fm_mean = torch.empty(self.p + 1, **f64)
        self.fm_t = torch.empty(self.p + 1, **f64)
        self.pool_g = torch.empty((1, p2, p2), **f64)
        self.pool_s = torch.empty((1, p2), **f64)
        self.pool_beta = torch.empty((1, self.p + 1), **f64)
        self.pool_n = torch.empty(1, **f64)
        self.pool_rank = torch.empty(1, **i32)
        self.pred = torch.full((T, lda), float("nan"), **f64)
        # rebalance dates: the test dates (the last calendar date carries no label -> no rows)
        rd = np.arange(self.t_test, T - 1, dtype=np.int32)
        self.rdates = torch.from_numpy(rd).to(dev)
        nd = len(rd)
        self.nd = nd
        self.reb = {
            "k": torch.empty(nd, **i32),
            "books": torch.full((nd, 2, MAX_BOOK), -1, **i32),
            "weights": torch.zeros((nd, 2, MAX_BOOK), **f64),
            "sums": torch.empty((nd, 4), **f64),
            "upos": torch.empty((nd, 2, 2, MAX_BOOK), **i32),
            "usize": torch.empty((nd, 2), **i64),
            "status": torch.empty(nd, **i32),
        }
        self.pnl = {"value": torch.empty(nd + 1, **f64), "turnover": torch.empty(nd, **f64),
                    "long_ret": torch.empty(nd, **f64), "short_ret": torch.empty(nd, **f64)}
        self.ctx = _lib.Context.get(dev.index)
        # the step's latency-critical chain runs on a high-priority stream; the test dates'
        # Grams + per-date solve + Fama-MacBeth (results nobody downstream reads) run on a
        # low-priority side stream, so the queue arbiter hands freed CU slots to the main chain
        # first (AFM_PIPE_PRIO=0: equal priority)
        import os
        prio = os.environ.get("AFM_PIPE_PRIO", "1") != "0"
        self.main = torch.cuda.Stream(device=dev, priority=-8 if prio else 0)
        self.side = torch.cuda.Stream(device=dev, priority=0)
        self.fork = os.environ.get("AFM_PIPE_FORK", "pooled")
        self.labels_at = os.environ.get("AFM_PIPE_LABELS", "after")

    def step(self, events: dict | None = None, only=None):
        """One pass of the hot path.  ``events``: optional {stage: (start, end)} CUDA events.
        ``only``: optional set of stage names to run (profiling; the others keep their last
        results)."""
        L = _lib.lib()
        P = _lib.ptr
        chk = _lib.check
        g, c = self.g, self.cfg
        T, lda, p = self.T, self.lda, self.p
        import torch
        caller = torch.cuda.current_stream(g.device)
        self.main.wait_stream(caller)
        self.side.wait_stream(caller)

        def mark(stage, which):
            if events is not None:
                events[stage][which].record()

        def on(stage):
            return only is None or stage in only

        with torch.cuda.stream(self.main):
            h = self.ctx.bind_stream()
            if on("factors"):
                mark("factors", 0)
                # label planes on the side stream, enqueued AFTER the factor kernel: its 236
                # workgroups are dispatched first and the labels take the 20 CUs they leave free
                # (A/B on MI355X: 28.50-28.62 vs 28.67-28.77 ms/step with the labels in the factor
                # call, AFM_PIPE_LABELS=main).  Enqueued before it, they slowed the latency-bound
                # factor kernel by more than their own time (2500-asset shard 5.5 -> 7.1 ms).
                lab = self.labels_at == "main"
                chk(L.afm_factors_f64(h, T, g.A, lda, P(g.close), P(g.volume),
                                      P(g.ret1d) if lab else None, P(g.excess) if lab else None,
                                      P(g.vbits), P(self.out), P(self.nanfree), P(self.finite)),
                    "factors")
                if not lab:
                    with torch.cuda.stream(self.side):
                        hs = self.ctx.bind_stream()
                        chk(L.afm_labels_f64(hs, T, lda, 0, T, P(g.excess), P(g.ret1d),
                                             P(g.vbits), P(self.out[TARGET]), P(self.out[TMR])),
                            "labels")
                    h = self.ctx.bind_stream()
                chk(L.afm_drop_last_obs_bits(h, T, lda, P(g.vbits), P(self.finite), P(self.rows)),
                    "label rows")
                if not lab:
                    self.main.wait_stream(self.side)           # the Grams read the target plane
                mark("factors", 1)
            tt = self.t_test
            if on("xs_gram"):                                  # train + valid dates
                mark("xs_gram", 0)
                chk(L.afm_xs_gram_f64(h, P(self.out), T * lda, lda, g.A, -1, P(self.cols), p,
                                      c.ycol, P(self.rows), 0, tt, P(self.gram), P(self.shift)),
                    "xs_gram")
                mark("xs_gram", 1)

            def side_chain():
                if on("xs_solve") or on("xs_gram_test"):
                    self.side.wait_stream(self.main)               # after the fork point
                    with torch.cuda.stream(self.side):
                        hs = self.ctx.bind_stream()
                        mark("xs_gram_test", 0)                    # test dates
                        chk(L.afm_xs_gram_f64(hs, P(self.out), T * lda, lda, g.A, -1,
                                              P(self.cols), p, c.ycol, P(self.rows), tt, T - tt,
                                              P(self.gram[tt:]), P(self.shift[tt:])),
                            "xs_gram_test")
                        mark("xs_gram_test", 1)
                        if on("xs_solve"):
                            mark("xs_solve", 0)
                            chk(L.afm_ols_solve_f64(hs, P(self.gram), P(self.shift), p, T, c.tol,
                                                    P(self.beta), P(self.nobs), P(self.rank)),
                                "ols_solve")
                            chk(L.afm_fama_macbeth_f64(hs, P(self.beta), P(self.rank), T, p + 1,
                                                       P(self.fm_mean), P(self.fm_t)),
                                "fama_macbeth")
                            mark("xs_solve", 1)

            # fork the side stream after the pooled solve (AFM_PIPE_FORK=gram: right after the
            # train+valid Grams): the pooled moments and the one-workgroup pooled solve then run
            # without the side stream's Gram workgroups on their CUs (A/B on MI355X: 28.6-28.7
            # vs 29.2-29.3 ms/step; AFM_PIPE_FORK=predict, after the predictions: the same time)
            if self.fork == "gram":
                side_chain()
                h = self.ctx.bind_stream()
            if on("pooled_ols"):
                mark("pooled_ols", 0)
                chk(L.afm_pool_moments_f64(h, P(self.gram), P(self.shift), p, self.t_test,
                                           P(self.pool_g), P(self.pool_s)), "pool")
                chk(L.afm_ols_solve_f64(h, P(self.pool_g), P(self.pool_s), p, 1, c.tol,
                                        P(self.pool_beta), P(self.pool_n), P(self.pool_rank)),
                    "pool_solve")
                mark("pooled_ols", 1)
            if self.fork == "pooled":
                side_chain()
                h = self.ctx.bind_stream()
            if on("predict"):
                mark("predict", 0)
                chk(L.afm_predict_f64(h, P(self.out), T * lda, lda, self.t_test, T - self.t_test,
                                      P(self.cols), p, P(self.pool_beta), 0, P(self.finite),
                                      c.ycol, P(self.pred)), "predict")
                mark("predict", 1)
            if self.fork == "predict":
                side_chain()
                h = self.ctx.bind_stream()
            if on("rebalance"):
                mark("rebalance", 0)
                r = self.reb
                chk(L.afm_rebalance_f64(h, T, g.A, lda, P(self.rdates), self.nd, P(self.pred),
                                        P(g.tbits), P(self.out[c.ycol]), P(g.vbits), 0, T,
                                        -1 if c.window is None else int(c.window), P(g.close),
                                        P(self.out[N_FACTORS - 1]), c.top_n, c.lo, c.hi,
                                        P(r["k"]), P(r["books"]), P(r["weights"]), P(r["sums"]),
                                        P(r["upos"]), P(r["usize"]), P(r["status"])), "rebalance")
                mark("rebalance", 1)
            if on("pnl"):
                mark("pnl", 0)
                r = self.reb
                q = self.pnl
                chk(L.afm_pnl_scan_f64(h, self.nd, P(r["k"]), P(r["books"]), P(r["sums"]),
                                       P(r["upos"]), P(r["usize"]), 100000000.0, c.rate,
                                       P(q["value"]), P(q["turnover"]), P(q["long_ret"]),
                                       P(q["short_ret"])), "pnl")
                mark("pnl", 1)
        caller.wait_stream(self.main)                      # the step ends when both are done
        caller.wait_stream(self.side)
        self.ctx.bind_stream()

    def summary(self) -> dict:
        """Host copies of the headline results (after a synchronize)."""
        v = self.pnl["value"].cpu().numpy()
        r = v[1:] / v[:-1] - 1
        return {"final_value": float(v[-1]), "sharpe": float(r.mean() / r.std(ddof=1)),
                "fm_mean": self.fm_mean.cpu().numpy(), "fm_t": self.fm_t.cpu().numpy(),
                "pooled_beta": self.pool_beta[0].cpu().numpy(),
                "ranks": self.rank.cpu().numpy(), "k": self.reb["k"].cpu().numpy(),
                "status": self.reb["status"].cpu().numpy()}

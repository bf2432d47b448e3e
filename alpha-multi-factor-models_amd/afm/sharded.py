"""The hot path on N GPUs, one process per GPU.

Partitioning (``scaling: strong`` -- the panel is fixed, N GPUs share it):

* **Assets** (64-asset blocks) for the factor build and the per-date partial Grams: pandas'
  rolling/ewm states carry rounding history from each asset's first day, so an exact factor
  panel needs each asset's whole series on one device (an asset shard is exact; a date shard
  would have to replay every running state from day 0).
* **Dates** (64-date blocks) for everything cross-sectional: the per-date Gram contraction runs
  over assets, so each date's per-rank partial moments travel to the date's owner in ONE
  ``all_to_all`` and are merged there (Chan, in rank order -- deterministic); solves, the pooled
  OLS blocks and the rebalance/KKT books then run on owned dates.
* All-gathers carry the small series: per-date betas (factor returns, for Fama-MacBeth), the
  pooled 64-date block moments (the same combination tree as one GPU), test-date predictions
  (the rebalance needs the whole cross-section) and the per-date rebalance results; every rank
  then runs the sequential PnL scan (microseconds per date).

Inputs are replicated: every rank builds the full input grid (the seeded generator, or its own
copy of the reference frame), so history / close / tmr planes need no exchange.

``Comm`` wraps torch.distributed: RCCL (backend "nccl") on device tensors; with backend "gloo"
tensors are staged through host memory (CPU tests, or several ranks sharing one GPU).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .factors import N_FACTORS
from .grid import PanelGrid
from .pipeline import PipelineConfig, STAGES
from .portfolio import MAX_BOOK

EXCHANGE_STAGES = STAGES + ("exchange",)


def block_range(n: int, world: int, rank: int, unit: int = 64):
    """[lo, hi) of ``rank``'s share of ``n`` items split in whole ``unit``-blocks (the last
    block may be short)."""
    nb = (n + unit - 1) // unit
    b0, b1 = nb * rank // world, nb * (rank + 1) // world
    return min(unit * b0, n), min(unit * b1, n)


def even_range(n: int, world: int, rank: int):
    return n * rank // world, n * (rank + 1) // world


class Comm:
    """Collectives of one process group (torch.distributed)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.host = dist.get_backend(group) == "gloo"

    def _stage(self, t):
        return t.cpu() if self.host else t

    def all_gather(self, t):
        """Equal-shape all-gather -> tensor [world, *t.shape] on t's device."""
        import torch
        src = self._stage(t.contiguous())
        out = torch.empty((self.world,) + tuple(src.shape), dtype=src.dtype, device=src.device)
        if self.host:
            parts = [torch.empty_like(src) for _ in range(self.world)]
            self.dist.all_gather(parts, src, group=self.group)
            out = torch.stack(parts)
        else:
            self.dist.all_gather_into_tensor(out, src, group=self.group)
        return out.to(t.device)

    def all_gather_packed(self, tensors):
        """Several equal-shape-per-rank tensors of any dtypes in ONE all-gather (their bytes
        concatenated) -> list of [world, *t.shape] tensors."""
        import torch
        flat = [t.contiguous().view(-1).view(torch.uint8) for t in tensors]
        sizes = [f.numel() for f in flat]
        g = self.all_gather(torch.cat(flat))                     # [world, total bytes]
        out, off = [], 0
        for t, n in zip(tensors, sizes):
            part = g[:, off:off + n].contiguous().view(t.dtype)
            out.append(part.view((self.world,) + tuple(t.shape)))
            off += n
        return out

    def all_to_all(self, inp, in_splits, out_splits):
        """all_to_all_single along dim 0 with explicit split sizes (rows)."""
        import torch
        src = self._stage(inp.contiguous())
        out = torch.empty((sum(out_splits),) + tuple(src.shape[1:]), dtype=src.dtype,
                          device=src.device)
        self.dist.all_to_all_single(out, src, output_split_sizes=list(out_splits),
                                    input_split_sizes=list(in_splits), group=self.group)
        return out.to(inp.device)

    def barrier(self):
        self.dist.barrier(group=self.group)


class ShardedPipeline:
    """``Pipeline.step()`` on one rank of N (same results up to the reassociation of the per-date
    moment merge: rel ~1e-15 on betas)."""

    def __init__(self, grid: PanelGrid, comm: Comm, cfg: PipelineConfig | None = None):
        import torch
        self.full = grid
        self.comm = comm
        self.cfg = cfg or PipelineConfig()
        c = self.cfg
        dev = grid.device
        W, r = comm.world, comm.rank
        T, A, lda = grid.T, grid.A, grid.lda
        self.T, self.A, self.lda = T, A, lda
        self.p = p = len(c.cols)
        self.p2 = p + 2
        self.t_valid = int(T * c.train_frac)
        self.t_test = int(T * (c.train_frac + c.valid_frac))
        f64 = dict(dtype=torch.float64, device=dev)
        i64 = dict(dtype=torch.int64, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        nch = (T + 63) // 64
        # ---- asset shards (64-asset blocks; the last block may be short) ----
        self.arange = [block_range(A, W, q) for q in range(W)]
        self.lda_q = [(hi - lo + 63) // 64 * 64 for lo, hi in self.arange]
        a0, a1 = self.arange[r]
        self.a0, self.A_r, self.lda_r = a0, a1 - a0, self.lda_q[r]
        sl = slice(a0, a0 + self.lda_r)
        self.loc = PanelGrid(dates=grid.dates, ids=grid.ids[a0:a1],
                             close=grid.close[:, sl].contiguous(),
                             volume=grid.volume[:, sl].contiguous(),
                             ret1d=grid.ret1d[:, sl].contiguous(),
                             excess=grid.excess[:, sl].contiguous(),
                             valid=grid.valid[:, sl].contiguous(),
                             vbits=grid.vbits[:, sl].contiguous())
        self.out = torch.empty((N_FACTORS, T, self.lda_r), **f64)
        self.nanfree = torch.zeros((nch, self.lda_r), **i64)
        self.finite = torch.zeros((nch, self.lda_r), **i64)
        self.rows = torch.zeros((nch, self.lda_r), **i64)
        self.cols = torch.as_tensor(np.asarray(c.cols, dtype=np.int32), device=dev)
        p2 = self.p2
        self.gram_r = torch.empty((T, p2, p2), **f64)           # partial moments, all dates
        self.shift_r = torch.empty((T, p2), **f64)
        # the Grams are exactly symmetric (gram_kernel writes both halves from one value): only
        # the upper triangle + the shift travel in the exchange (half the bytes)
        iu = torch.triu_indices(p2, p2)
        self.tri = (iu[0] * p2 + iu[1]).to(dev)
        self.tri_t = (iu[1] * p2 + iu[0]).to(dev)
        self.ntri = int(self.tri.numel())
        # ---- date shards (64-date blocks) ----
        self.drange = [block_range(T, W, q) for q in range(W)]
        d0, d1 = self.drange[r]
        self.d0, self.nd_own = d0, d1 - d0
        self.nd_q = [hi - lo for lo, hi in self.drange]
        self.nd_max = max(self.nd_q)
        self.gram = torch.empty((max(self.nd_own, 1), p2, p2), **f64)   # merged, owned dates
        self.shift = torch.empty((max(self.nd_own, 1), p2), **f64)
        self.beta_own = torch.full((self.nd_max, p + 1), float("nan"), **f64)
        self.nobs_own = torch.zeros(self.nd_max, **f64)
        self.rank_own = torch.zeros(self.nd_max, **i32)
        self.beta = torch.empty((T, p + 1), **f64)
        self.nobs = torch.empty(T, **f64)
        self.rank = torch.empty(T, **i32)
        self.fm_mean = torch.empty(p + 1, **f64)
        self.fm_t = torch.empty(p + 1, **f64)
        # pooled OLS over [0, t_test): 64-date blocks of the owned dates
        self.ntr_q = [max(0, min(self.t_test, hi) - lo) for lo, hi in self.drange]
        self.nb_q = [(n + 63) // 64 for n in self.ntr_q]
        self.nb_max = max(max(self.nb_q), 1)
        self.blk_g = torch.zeros((self.nb_max, p2, p2), **f64)
        self.blk_s = torch.zeros((self.nb_max, p2), **f64)
        self.blk16_g = torch.zeros((4 * self.nb_max, p2, p2), **f64)     # tree level 0 results
        self.blk16_s = torch.zeros((4 * self.nb_max, p2), **f64)
        # the gathered [W][nb_max] blocks without the padding: the 64-date blocks in date order
        self.blk_idx = torch.as_tensor(np.concatenate(
            [q * self.nb_max + np.arange(self.nb_q[q]) for q in range(W)]).astype(np.int64),
            device=dev)
        self.pool_g = torch.empty((1, p2, p2), **f64)
        self.pool_s = torch.empty((1, p2), **f64)
        self.pool_beta = torch.empty((1, p + 1), **f64)
        self.pool_n = torch.empty(1, **f64)
        self.pool_rank = torch.empty(1, **i32)
        # predictions: local slice, then the whole cross-section of the test dates
        self.pred_r = torch.full((T, self.lda_r), float("nan"), **f64)
        self.lda_max = max(self.lda_q)
        self.pred = torch.full((T, lda), float("nan"), **f64)
        # label planes for every asset over the dates the rebalance reads
        self.target = torch.full((T, lda), float("nan"), **f64)
        self.tmr = torch.full((T, lda), float("nan"), **f64)
        win = c.window if c.window is not None else T
        self.lab0 = max(0, self.t_test - int(win) - 1) if c.window is not None else 0
        # rebalance dates, split evenly; each rank runs its share plus one neighbour per side
        rd = np.arange(self.t_test, T - 1, dtype=np.int32)
        self.nd = nd = len(rd)
        self.rrange = [even_range(nd, W, q) for q in range(W)]
        i0, i1 = self.rrange[r]
        self.i0, self.i1 = i0, i1
        self.e0, self.e1 = max(i0 - 1, 0), min(i1 + 1, nd)
        self.rd_ext = torch.from_numpy(rd[self.e0:self.e1].copy()).to(dev)
        ne = max(self.e1 - self.e0, 1)
        self.reb_ext = {
            "k": torch.zeros(ne, **i32),
            "books": torch.full((ne, 2, MAX_BOOK), -1, **i32),
            "weights": torch.zeros((ne, 2, MAX_BOOK), **f64),
            "sums": torch.zeros((ne, 4), **f64),
            "upos": torch.full((ne, 2, 2, MAX_BOOK), -1, **i32),
            "usize": torch.zeros((ne, 2), **i64),
            "status": torch.zeros(ne, **i32),
        }
        self.nr_max = max(hi - lo for lo, hi in self.rrange)
        self.reb = {k: torch.zeros((nd,) + tuple(v.shape[1:]), dtype=v.dtype, device=dev)
                    for k, v in self.reb_ext.items()}
        self.pnl = {"value": torch.empty(nd + 1, **f64), "turnover": torch.empty(nd, **f64),
                    "long_ret": torch.empty(nd, **f64), "short_ret": torch.empty(nd, **f64)}
        self.ctx = _lib.Context.get(dev.index)
        # side stream: the full-width label planes (overlapping the exchange) and the per-date
        # solve of the owned dates (nothing on the main chain reads the betas)
        self.side = torch.cuda.Stream(device=dev)

    def n_asset_days_local(self) -> int:
        return int(self.loc.valid.sum().item())

    # ------------------------------------------------------------------------------------------
    def step(self, events: dict | None = None):
        import torch
        L = _lib.lib()
        P = _lib.ptr
        chk = _lib.check
        c = self.cfg
        cm = self.comm
        T, lda, p, p2 = self.T, self.lda, self.p, self.p2
        lr = self.lda_r
        h = self.ctx.bind_stream()

        def mark(stage, which):
            if events is not None:
                events[stage][which].record()

        g = self.loc
        f = self.full
        main = torch.cuda.current_stream(self.out.device)
        side = self.side
        side.wait_stream(main)
        mark("factors", 0)
        chk(L.afm_factors_f64(h, T, self.A_r, lr, P(g.close), P(g.volume), P(g.ret1d),
                              P(g.excess), P(g.vbits), P(self.out), P(self.nanfree),
                              P(self.finite)), "factors")
        chk(L.afm_drop_last_obs_bits(h, T, lr, P(g.vbits), P(self.finite), P(self.rows)),
            "label rows")
        mark("factors", 1)
        mark("xs_gram", 0)
        chk(L.afm_xs_gram_f64(h, P(self.out), T * lr, lr, self.A_r, -1, P(self.cols), p, c.ycol,
                              P(self.rows), 0, T, P(self.gram_r), P(self.shift_r)), "xs_gram")
        mark("xs_gram", 1)
        # history label planes (all assets, read by the rebalance) on the side stream, overlapping
        # the exchange; next to the latency-bound factor kernel they would slow it (A/B: 2500
        # assets 5.5 -> 7.1 ms)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            hs = self.ctx.bind_stream()
            chk(L.afm_labels_f64(hs, T, lda, self.lab0, T, P(f.excess), P(f.ret1d), P(f.vbits),
                                 P(self.target), P(self.tmr)), "labels")
            labels_done = torch.cuda.Event()
            labels_done.record(side)
        h = self.ctx.bind_stream()
        # ---- exchange: each date's per-rank partial moments -> the date's owner ----
        mark("exchange", 0)
        W = cm.world
        send = torch.cat([self.gram_r.view(T, p2 * p2).index_select(1, self.tri), self.shift_r],
                         dim=1)
        recv = cm.all_to_all(send, self.nd_q, [self.nd_own] * W)  # [W * nd_own][ntri + p2]
        rs = recv[:, self.ntri:]
        rg = torch.empty((recv.shape[0], p2 * p2), dtype=recv.dtype, device=recv.device)
        rg[:, self.tri] = recv[:, :self.ntri]
        rg[:, self.tri_t] = recv[:, :self.ntri]
        mark("exchange", 1)
        h = self.ctx.bind_stream()
        if self.nd_own > 0:
            rg = rg.view(W, self.nd_own, p2 * p2).transpose(0, 1).contiguous()   # [date][rank]
            rs = rs.view(W, self.nd_own, p2).transpose(0, 1).contiguous()
            chk(L.afm_pool_segments_f64(h, P(rg), P(rs), p, self.nd_own * W, W, P(self.gram),
                                        P(self.shift)), "merge partial moments")
        # per-date solve of the owned dates on the side stream; its beta all-gather + Fama-MacBeth
        # are issued after the main chain's collectives (one RCCL stream serialises collectives
        # in issue order, so issuing it here would hold the pooled-OLS gather behind the solve)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            hs = self.ctx.bind_stream()
            mark("xs_solve", 0)
            if self.nd_own > 0:
                chk(L.afm_ols_solve_f64(hs, P(self.gram), P(self.shift), p, self.nd_own, c.tol,
                                        P(self.beta_own), P(self.nobs_own), P(self.rank_own)),
                    "ols_solve")
        h = self.ctx.bind_stream()
        # ---- pooled OLS over [0, t_test): owned 64-date blocks, gathered in date order, then the
        # rest of afm_pool_moments_f64's tree (the same tree as one device: bit-identical) ----
        mark("pooled_ols", 0)
        ntr = self.ntr_q[cm.rank]
        self.blk_g.zero_()
        self.blk_s.zero_()
        if ntr > 0:                                   # tree levels 0-1 (afm_pool_tree_f64)
            n16 = (ntr + 15) // 16
            chk(L.afm_pool_segments_f64(h, P(self.gram), P(self.shift), p, ntr, 16,
                                        P(self.blk16_g), P(self.blk16_s)), "pool 16-date blocks")
            chk(L.afm_pool_segments_f64(h, P(self.blk16_g), P(self.blk16_s), p, n16, 4,
                                        P(self.blk_g), P(self.blk_s)), "pool 64-date blocks")
        ag, as_ = cm.all_gather_packed([self.blk_g, self.blk_s])
        ag = ag.reshape(W * self.nb_max, p2, p2).index_select(0, self.blk_idx).contiguous()
        as_ = as_.reshape(W * self.nb_max, p2).index_select(0, self.blk_idx).contiguous()
        h = self.ctx.bind_stream()
        chk(L.afm_pool_tree_f64(h, P(ag), P(as_), p, int(self.blk_idx.numel()), 2,
                                P(self.pool_g), P(self.pool_s)), "pool")
        chk(L.afm_ols_solve_f64(h, P(self.pool_g), P(self.pool_s), p, 1, c.tol,
                                P(self.pool_beta), P(self.pool_n), P(self.pool_rank)),
            "pool_solve")
        mark("pooled_ols", 1)
        # ---- predictions on the test dates: local slice, then the whole cross-section ----
        mark("predict", 0)
        nt = T - self.t_test
        chk(L.afm_predict_f64(h, P(self.out), T * lr, lr, self.t_test, nt, P(self.cols), p,
                              P(self.pool_beta), 0, P(self.finite), c.ycol, P(self.pred_r)),
            "predict")
        pr = self.pred_r[self.t_test:]
        if lr < self.lda_max:
            pr = torch.nn.functional.pad(pr, (0, self.lda_max - lr), value=float("nan"))
        pg = cm.all_gather(pr)
        for q, (lo, hi) in enumerate(self.arange):
            self.pred[self.t_test:, lo:lo + self.lda_q[q]] = pg[q, :, :self.lda_q[q]]
        mark("predict", 1)
        # ---- rebalance + KKT on the owned rebalance dates (+ one neighbour per side) ----
        main.wait_event(labels_done)                   # history planes
        h = self.ctx.bind_stream()
        mark("rebalance", 0)
        x = self.reb_ext
        ne = self.e1 - self.e0
        if ne > 0:
            chk(L.afm_rebalance_f64(h, T, self.A, lda, P(self.rd_ext), ne, P(self.pred),
                                    P(f.tbits), P(self.target), P(f.vbits), 0, T,
                                    -1 if c.window is None else int(c.window), P(f.close),
                                    P(self.tmr), c.top_n, c.lo, c.hi, P(x["k"]), P(x["books"]),
                                    P(x["weights"]), P(x["sums"]), P(x["upos"]), P(x["usize"]),
                                    P(x["status"])), "rebalance")
        lo = self.i0 - self.e0
        n_own = self.i1 - self.i0
        owns = []
        for k, v in x.items():
            own = v[lo:lo + n_own]
            if n_own < self.nr_max:
                pad = torch.zeros((self.nr_max - n_own,) + tuple(v.shape[1:]), dtype=v.dtype,
                                  device=v.device)
                own = torch.cat([own, pad])
            owns.append(own)
        for k, gath in zip(x.keys(), cm.all_gather_packed(owns)):    # one collective
            for q, (qlo, qhi) in enumerate(self.rrange):
                self.reb[k][qlo:qhi] = gath[q, :qhi - qlo]
        mark("rebalance", 1)
        h = self.ctx.bind_stream()
        mark("pnl", 0)
        r, q_ = self.reb, self.pnl
        chk(L.afm_pnl_scan_f64(h, self.nd, P(r["k"]), P(r["books"]), P(r["sums"]), P(r["upos"]),
                               P(r["usize"]), 100000000.0, c.rate, P(q_["value"]),
                               P(q_["turnover"]), P(q_["long_ret"]), P(q_["short_ret"])), "pnl")
        mark("pnl", 1)
        # ---- per-date betas -> every rank, Fama-MacBeth (side stream, overlaps the PnL scan) ----
        with torch.cuda.stream(side):
            bg, ng, kg = cm.all_gather_packed([self.beta_own, self.nobs_own, self.rank_own])
            for q, (lo, hi) in enumerate(self.drange):
                self.beta[lo:hi] = bg[q, :hi - lo]
                self.nobs[lo:hi] = ng[q, :hi - lo]
                self.rank[lo:hi] = kg[q, :hi - lo]
            hs = self.ctx.bind_stream()
            chk(L.afm_fama_macbeth_f64(hs, P(self.beta), P(self.rank), T, p + 1, P(self.fm_mean),
                                       P(self.fm_t)), "fama_macbeth")
            mark("xs_solve", 1)
        main.wait_stream(side)                         # the step ends when both are done
        self.ctx.bind_stream()

    def summary(self) -> dict:
        v = self.pnl["value"].cpu().numpy()
        rr = v[1:] / v[:-1] - 1
        return {"final_value": float(v[-1]), "sharpe": float(rr.mean() / rr.std(ddof=1)),
                "fm_mean": self.fm_mean.cpu().numpy(), "fm_t": self.fm_t.cpu().numpy(),
                "pooled_beta": self.pool_beta[0].cpu().numpy(),
                "ranks": self.rank.cpu().numpy(), "k": self.reb["k"].cpu().numpy(),
                "status": self.reb["status"].cpu().numpy()}

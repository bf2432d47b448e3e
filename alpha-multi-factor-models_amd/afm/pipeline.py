"""The reference's hot path, end to end on one device (BASELINE.json ``metric``; SURVEY.md §8(a)
rows I0-I16, A1-A4, R1, K1-K4): the notebook chain that feeds ``PortfolioManager``.

One ``step()`` over a device-resident calendar-grid panel:

1. factors      afm_factors_f64: the 98 No-talib.py columns (NT:1-93); all_df rows = the NT:33
                dropna rows (label planes non-NaN)
2. zstats       train-window per-security mean / std of the 97 feature columns (KKT:424-451:
                train = dates <= train_end, features = Index.difference order, KKT:433-443 --
                tmr_ret1d included, as in the reference); assets with a non-finite mean or a
                zero / NaN std drop out entirely (their z is NaN in every row, KKT:452-454)
3. xs_gram      the pooled Gram of [1, z_1..z_97, target] over every train + valid row, on fp64
                MFMA with z computed on the fly (afm_zpool_f64: one partial per 64-asset row-block
                and date chunk, summed over a fixed tree -- row-blocks within the 8 asset blocks,
                then the blocks -- so it is bit-identical for any GPU count).  The inclusive
                .loc slices of KKT:426-427 put train_end in train AND valid: its Gram is added
                once more.
4. lasso        Lasso(alpha=2e-4, max_iter=10000).fit (KKT:605-607) by Gram coordinate descent
5. predict      lasso.predict on the test dates (KKT:612), z on the fly
6. rebalance    PortfolioManager(lasso_predict, ...).calculate_portfolio() (KKT:976-977):
                per test date top/bottom-n books, rolling-window pairwise covariance of the
                target history (north star: 252 dates; None = the reference's whole
                training window), exact box-QP weights (SLSQP's problem, KKT:811-833)
7. pnl          value / turnover recursion (KKT:864-892)
side streams:
8. analyzer     AlphaSignalAnalyzer(lasso_predict, price_data=df_test close).run() (KKT:630-631):
                forward returns, IC, decile layers, top-10 backtest, IR
9. fm           the north-star extension: classic Fama-MacBeth -- per-date Grams of
                [1, FM30 factor values, target] over the same rows (afm_zgram_f64: per (date,
                asset block) partials, fixed tree), per-date cross-sectional OLS, mean / t.
                FM30 is a stated well-conditioned subset of the 97 features (worst date
                cond(corr) ~3e2 on config A, raw or z-scored).

The reference's LinearRegression over all 97 columns (KKT:582-583) is not a stage: that design
is numerically rank-deficient (cond ~1e10 measured on config A: BBANDS_upper + BBANDS_lower =
2 SMA before z-scoring, and the price-level columns are nearly collinear after), so its
coefficients carry ~1e-6 relative noise even in scikit-learn's SVD solve and no implementation
can be checked against another.  The portfolio consumes the Lasso predictions (KKT:976) --
a well-posed fit -- and that chain is what a step runs.  ``afm.LinearRegression`` remains the
drop-in for well-conditioned designs.

All buffers are allocated once; a step does no host synchronisation.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

from . import _lib
from .factors import COL, FACTOR_NAMES, N_FACTORS, TARGET, TMR
from .grid import PanelGrid
from .portfolio import MAX_BOOK

# KKT:433-443: every column except the raw inputs and `target`, in Index.difference (sorted)
# order -- the 96 factors and tmr_ret1d
FEATURES = sorted(n for n in FACTOR_NAMES if n != "target")
# Fama-MacBeth design (the north-star per-date regression): 30 z-scored columns chosen greedily
# for the smallest worst-date condition number on the config-A synthetic panel (worst sampled
# date cond(corr) ~ 3e2; the full 97-column design is ~1e10 pooled, singular per date)
FM30 = ["tmr_ret1d", "ACCEL_32", "sd5_15", "corr_5", "OBV", "sd_15", "MOM_38", "volsd5_15",
        "vol_change", "volsd_15", "corr_15", "ACCEL_38", "BBANDS_upper_14", "ACCEL_20",
        "ACCEL_26", "ROCR_14", "sd_3", "ACCEL_50", "volsd_3", "ACCEL_44", "ACCEL_56", "ROCR_20",
        "ROCR_56", "PVT", "PSY", "ROCR_32", "MOM_26", "ACCEL_14", "RSI_8", "MOM_50"]
N_BLOCKS = 8           # fixed asset blocks of the Gram trees (>= the largest GPU count)
N_CHUNKS = 16          # date chunks of the pooled Gram's row-block partials

STAGES = ("factors", "zstats", "xs_gram", "lasso", "predict", "rebalance", "pnl", "fm",
          "analyzer")
PIPELINE_STAGES = STAGES


@dataclass
class PipelineConfig:
    train_end: str = "2015-12-31"   # KKT:424
    valid_end: str = "2016-12-31"   # KKT:425
    alpha: float = 2e-4             # KKT:605
    max_iter: int = 10000           # KKT:605
    lasso_tol: float = 1e-4         # sklearn Lasso default
    fm_features: tuple = tuple(FM30)
    top_n: int = 10                 # KKT:796
    window: int | None = 252        # rolling covariance window (north star); None = KKT:858
    lo: float = 0.0                 # KKT:828
    hi: float = 0.1
    rate: float = 1e-4              # KKT:796
    v0: float = 100000000.0         # KKT:804
    tol: float = 1e-10              # pivot threshold of the per-date solve
    analyzer: bool = True


@dataclass
class Split:
    """The reference's date split on the calendar (KKT:424-428): ``.loc`` slices are inclusive at
    both ends.  train = [0, tr1), valid = [v0, v1), test = [s0, T); ``dup``: train_end is a
    trading date, so it is in train AND valid (its rows enter the fit twice)."""
    tr1: int
    v0: int
    v1: int
    s0: int
    dup: bool

    @classmethod
    def of(cls, dates, train_end, valid_end) -> "Split":
        d = np.asarray(dates).astype("datetime64[ns]")
        te = np.datetime64(np.datetime64(train_end, "D"), "ns")
        ve = np.datetime64(np.datetime64(valid_end, "D"), "ns")
        tr1 = int(np.searchsorted(d, te, side="right"))
        v0 = int(np.searchsorted(d, te, side="left"))
        v1 = int(np.searchsorted(d, ve, side="right"))
        s0 = int(np.searchsorted(d, ve, side="left"))
        if tr1 < 2 or s0 >= len(d) - 1 or v1 <= v0:
            raise ValueError(f"split {train_end} / {valid_end} leaves an empty train, valid or "
                             f"test range on {d[0]} .. {d[-1]}")
        return cls(tr1, v0, v1, s0, bool(v0 < tr1))


def block_assets(lda: int, nblk: int = N_BLOCKS) -> int:
    """Assets per Gram block: the 64-asset groups split into nblk equal runs."""
    return max(1, -(-(lda // 64) // nblk)) * 64


class Pipeline:
    def __init__(self, grid: PanelGrid, cfg: PipelineConfig | None = None):
        import torch
        self.g = grid
        self.cfg = c = cfg or PipelineConfig()
        dev = grid.device
        T, lda, A = grid.T, grid.lda, grid.A
        nch = (T + 63) // 64
        self.T, self.lda, self.A = T, lda, A
        self.sp = sp = Split.of(grid.dates, c.train_end, c.valid_end)
        self.p = p = len(FEATURES)
        self.p2 = p + 2
        f64 = dict(dtype=torch.float64, device=dev)
        i64 = dict(dtype=torch.int64, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        self.feat = torch.as_tensor(np.array([COL[n] for n in FEATURES], np.int32), device=dev)
        self.pf = len(c.fm_features)
        self.out = torch.full((N_FACTORS, T, lda), float("nan"), **f64)
        self.nanfree = torch.zeros((nch, lda), **i64)
        self.finite = torch.zeros((nch, lda), **i64)
        self.alldf = torch.zeros((nch, lda), **i64)      # all_df rows (NT:33 dropna)
        self.frows = torch.zeros((nch, lda), **i64)      # all_df rows with every feature finite
        self.zrows = torch.zeros((nch, lda), **i64)      # rows surviving the z-score dropna
        self.mu = torch.empty((p, lda), **f64)
        self.sd = torch.empty((p, lda), **f64)
        self.zs = torch.empty((p + 1, lda, 2), **f64)
        self.asset_ok = torch.empty(lda, **i32)
        self.nblk = N_BLOCKS
        self.blk = block_assets(lda)
        self.nrb = (A + 63) // 64                        # 64-asset row-blocks
        self.rb_per_blk = self.blk // 64
        L = _lib.lib()
        pe = L.afm_zgram_part_bytes(p) // 8
        self.pool_part = torch.empty((self.nrb, N_CHUNKS, pe), **f64)
        self.pool_rb = torch.empty((self.nrb, pe), **f64)
        self.pool_blk = torch.empty((self.nblk, pe), **f64)
        self.pool_g = torch.empty((1, self.p2, self.p2), **f64)
        self.pool_s = torch.zeros((1, self.p2), **f64)   # raw moments: zero shift
        self.te_part = torch.empty((self.nblk, pe), **f64)
        self.te_gram = torch.empty((1, self.p2, self.p2), **f64)
        self.lasso_beta = torch.empty(p + 1, **f64)
        self.lasso_info = torch.empty(3, **f64)
        # FM design: [1, FM30 z-scores, target] per date
        self.fm_cols = torch.as_tensor(np.array([COL[n] for n in c.fm_features], np.int32),
                                       device=dev)
        pef = L.afm_zgram_part_bytes(self.pf) // 8
        self.fm_part = torch.empty((T, self.nblk, pef), **f64)
        self.fm_gram = torch.empty((T, self.pf + 2, self.pf + 2), **f64)
        self.fm_shift = torch.zeros((T, self.pf + 2), **f64)
        self.pred = torch.full((T, lda), float("nan"), **f64)
        self.fm_beta = torch.empty((T, self.pf + 1), **f64)
        self.fm_nobs = torch.empty(T, **f64)
        self.fm_rank = torch.empty(T, **i32)
        self.fm_mean = torch.empty(self.pf + 1, **f64)
        self.fm_t = torch.empty(self.pf + 1, **f64)
        # rebalance dates: the test dates that can carry predictions (a present observation that
        # is not the asset's last -- every other row lacks the target)
        vb = grid.valid.cpu().numpy() if hasattr(grid.valid, "cpu") else np.asarray(grid.valid)
        nxt = np.zeros_like(vb)
        nxt[:-1] = np.flip(np.logical_or.accumulate(np.flip(vb[1:], 0), 0), 0)
        has = (vb & nxt).any(axis=1)
        rd = np.flatnonzero(has[sp.s0:]).astype(np.int32) + sp.s0
        self.rdates = torch.from_numpy(rd).to(dev)
        self.nd = nd = len(rd)
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
        # analyzer on the test sub-grid (64-date aligned, so the bit words line up)
        self.a0 = (sp.s0 // 64) * 64
        Ta = T - self.a0
        self.Ta = Ta
        self.price_bits = torch.zeros((nch, lda), **i64)  # df_test rows (all_df, date >= valid_end)
        if c.analyzer:
            self.an = {
                "fr": torch.empty((3, Ta, lda), **f64),
                "scratch": torch.empty((Ta, lda), **f64),
                "rows": torch.empty((4, Ta, lda), **f64),
                "rows_idx": torch.empty((Ta, lda), **i32),
                "nrows": torch.empty(Ta, **i32),
                "skey": torch.empty((Ta, lda), **i64),
                "sidx": torch.empty((Ta, lda), **i32),
                "ra": torch.empty((Ta, lda), **i32),
                "rd": torch.empty((Ta, lda), **i32),
            }
            ad = np.arange(sp.s0 - self.a0, Ta, dtype=np.int32)    # test dates, sub-grid index
            self.an_dates = torch.from_numpy(ad).to(dev)
            self.an_nd = nad = len(ad)
            years = np.asarray(grid.dates).astype("datetime64[Y]").astype(np.int64) + 1970
            yr = years[self.a0 + ad].astype(np.int32)
            self.an_year0, self.an_nyears = int(yr.min()), int(yr.max() - yr.min() + 1)
            self.an_year = torch.from_numpy(yr).to(dev)
            self.an.update({
                "ic": torch.empty((nad, 3), **f64),
                "layer_mean": torch.empty((nad, 3, 10), **f64),
                "layer_cnt": torch.empty((nad, 10), **i32),
                "port": torch.empty((nad, 3), **f64),
                "cum_layer": torch.empty((nad, 3, 10), **f64),
                "ls": torch.empty((nad, 3, 5), **f64),
                "cum_port": torch.empty((nad, 3), **f64),
                "ir": torch.empty((self.an_nyears, 3), **f64),
                "ir_scratch": torch.empty((3 * self.an_nyears, nad), **f64),
            })
        self.ctx = _lib.Context.get(dev.index)
        prio = os.environ.get("AFM_PIPE_PRIO", "1") != "0"
        self.main = torch.cuda.Stream(device=dev, priority=-8 if prio else 0)
        self.side = torch.cuda.Stream(device=dev, priority=0)
        self.side2 = torch.cuda.Stream(device=dev, priority=0)

    # ------------------------------------------------------------------------------------------
    def _pooled_gram(self, h, t0, nt):
        """Pooled Gram of the rows of the dates [t0, t0 + nt): row-block x chunk partials, then
        the tree (chunks of a row-block, row-blocks of an asset block, the asset blocks)."""
        L, P, chk = _lib.lib(), _lib.ptr, _lib.check
        T, lda, p = self.T, self.lda, self.p
        chk(L.afm_zpool_f64(h, P(self.out), T * lda, lda, P(self.feat), None, p, TARGET,
                            P(self.zs), p, P(self.zrows), t0, nt, 0, self.nrb, self.A, N_CHUNKS,
                            P(self.pool_part), 0), "zpool")
        chk(L.afm_gram_tree_f64(h, p, P(self.pool_part), self.nrb * N_CHUNKS, N_CHUNKS, 0,
                                P(self.pool_rb)), "tree chunks")
        chk(L.afm_gram_tree_f64(h, p, P(self.pool_rb), self.nrb, self.rb_per_blk, 0,
                                P(self.pool_blk)), "tree row-blocks")
        nb = -(-self.nrb // self.rb_per_blk)
        chk(L.afm_gram_tree_f64(h, p, P(self.pool_blk), nb, self.nblk, 1, P(self.pool_g)),
            "tree blocks")

    def _date_gram(self, h, t, part, gram):
        """The full Gram of one date (the train_end duplicate)."""
        L, P, chk = _lib.lib(), _lib.ptr, _lib.check
        T, lda, p = self.T, self.lda, self.p
        chk(L.afm_zgram_f64(h, P(self.out), T * lda, lda, P(self.feat), None, p, TARGET,
                            P(self.zs), p, P(self.zrows), t, 1, self.nblk, 0, self.blk, self.A,
                            P(part), 0), "zgram date")
        chk(L.afm_gram_tree_f64(h, p, P(part), self.nblk, self.nblk, 1, P(gram)), "tree date")

    def _fm(self, h):
        """Per-date FM30 Grams, solves and Fama-MacBeth statistics."""
        L, P, chk = _lib.lib(), _lib.ptr, _lib.check
        T, lda, p, pf, c = self.T, self.lda, self.p, self.pf, self.cfg
        chk(L.afm_zgram_f64(h, P(self.out), T * lda, lda, P(self.fm_cols), None, pf, TARGET,
                            None, 0, P(self.zrows), 0, T, self.nblk, 0, self.blk, self.A,
                            P(self.fm_part), 0), "zgram fm")
        chk(L.afm_gram_tree_f64(h, pf, P(self.fm_part), T * self.nblk, self.nblk, 1,
                                P(self.fm_gram)), "tree fm")
        chk(L.afm_ols_solve_f64(h, P(self.fm_gram), P(self.fm_shift), pf, T, c.tol,
                                P(self.fm_beta), P(self.fm_nobs), P(self.fm_rank)), "fm solve")
        chk(L.afm_fama_macbeth_f64(h, P(self.fm_beta), P(self.fm_rank), T, pf + 1,
                                   P(self.fm_mean), P(self.fm_t)), "fama_macbeth")

    def step(self, events: dict | None = None):
        """One pass of the chain.  ``events``: optional {stage: (start, end)} CUDA events."""
        import torch
        L, P, chk = _lib.lib(), _lib.ptr, _lib.check
        g, c, sp = self.g, self.cfg, self.sp
        T, lda, p = self.T, self.lda, self.p
        nch = (T + 63) // 64
        caller = torch.cuda.current_stream(g.device)
        for s in (self.main, self.side, self.side2):
            s.wait_stream(caller)

        def mark(stage, which):
            if events is not None and stage in events:
                events[stage][which].record()

        with torch.cuda.stream(self.main):
            h = self.ctx.bind_stream()
            mark("factors", 0)
            chk(L.afm_factors_f64(h, T, g.A, lda, P(g.close), P(g.volume), P(g.ret1d),
                                  P(g.excess), P(g.vbits), P(self.out), P(self.nanfree),
                                  P(self.finite)), "factors")
            chk(L.afm_drop_last_obs_bits(h, T, lda, P(g.vbits), P(self.nanfree), P(self.alldf)),
                "all_df rows")
            chk(L.afm_drop_last_obs_bits(h, T, lda, P(g.vbits), P(self.finite), P(self.frows)),
                "finite rows")
            mark("factors", 1)
            mark("zstats", 0)
            chk(L.afm_zscore_stats_f64(h, P(self.out), T * lda, T, lda, P(self.feat), p,
                                       P(self.alldf), 0, sp.tr1, P(self.mu), P(self.sd)),
                "zscore stats")
            chk(L.afm_zstats_finalize_f64(h, P(self.mu), P(self.sd), p, lda, P(self.zs),
                                          P(self.asset_ok)), "zstats finalize")
            chk(L.afm_row_bits(h, nch, lda, P(self.frows), None, P(self.asset_ok), 0, T,
                               P(self.zrows)), "z rows")
            mark("zstats", 1)
            # side stream: the per-date FM30 regressions (nothing downstream reads them)
            self.side.wait_stream(self.main)
            with torch.cuda.stream(self.side):
                hs = self.ctx.bind_stream()
                mark("fm", 0)
                self._fm(hs)
                mark("fm", 1)
            h = self.ctx.bind_stream()
            mark("xs_gram", 0)
            self._pooled_gram(h, 0, sp.v1)                          # train + valid rows
            if sp.dup:                                              # train_end counted twice
                self._date_gram(h, sp.tr1 - 1, self.te_part, self.te_gram)
                chk(L.afm_vec_add_f64(h, self.p2 * self.p2, P(self.te_gram), P(self.pool_g)),
                    "dup")
            mark("xs_gram", 1)
            mark("lasso", 0)
            chk(L.afm_lasso_fit_f64(h, P(self.pool_g), P(self.pool_s), p, c.alpha, c.max_iter,
                                    c.lasso_tol, 0, P(self.lasso_beta), P(self.lasso_info)),
                "lasso")
            mark("lasso", 1)
            mark("predict", 0)
            chk(L.afm_zpredict_f64(h, P(self.out), T * lda, lda, sp.s0, T - sp.s0, P(self.feat),
                                   p, P(self.zs), P(self.lasso_beta), P(self.zrows),
                                   P(self.pred)), "predict")
            mark("predict", 1)
            if c.analyzer:
                self.side2.wait_stream(self.main)
                with torch.cuda.stream(self.side2):
                    self._analyzer(mark)
                h = self.ctx.bind_stream()
            mark("rebalance", 0)
            r = self.reb
            chk(L.afm_rebalance_f64(h, T, g.A, lda, P(self.rdates), self.nd, P(self.pred),
                                    P(g.tbits), P(self.out[TARGET]), P(self.zrows), 0, sp.tr1,
                                    -1 if c.window is None else int(c.window), P(g.close),
                                    P(self.out[TMR]), c.top_n, c.lo, c.hi, P(r["k"]),
                                    P(r["books"]), P(r["weights"]), P(r["sums"]), P(r["upos"]),
                                    P(r["usize"]), P(r["status"])), "rebalance")
            mark("rebalance", 1)
            mark("pnl", 0)
            q = self.pnl
            chk(L.afm_pnl_scan_f64(h, self.nd, P(r["k"]), P(r["books"]), P(r["sums"]),
                                   P(r["upos"]), P(r["usize"]), c.v0, c.rate, P(q["value"]),
                                   P(q["turnover"]), P(q["long_ret"]), P(q["short_ret"])), "pnl")
            mark("pnl", 1)
        for s in (self.main, self.side, self.side2):
            caller.wait_stream(s)
        self.ctx.bind_stream()

    def _analyzer(self, mark):
        """AlphaSignalAnalyzer(lasso_predict, price_data=df_test[['close_price']]).run()
        (KKT:630-631) on the test sub-grid, no host synchronisation."""
        L, P, chk = _lib.lib(), _lib.ptr, _lib.check
        g, sp, an = self.g, self.sp, self.an
        T, lda, a0, Ta = self.T, self.lda, self.a0, self.Ta
        nch = (T + 63) // 64
        h = self.ctx.bind_stream()
        mark("analyzer", 0)
        chk(L.afm_row_bits(h, nch, lda, P(self.alldf), None, None, sp.s0, T, P(self.price_bits)),
            "price rows")
        cb = a0 // 64
        chk(L.afm_fwd_returns_f64(h, Ta, lda, P(g.close[a0:]), P(self.price_bits[cb:]),
                                  P(an["fr"])), "fwd_returns")
        chk(L.afm_xs_prepare_f64(h, Ta, g.A, lda, P(self.pred[a0:]), P(an["fr"]),
                                 P(an["scratch"]), P(an["rows"]), P(an["rows_idx"]),
                                 P(an["nrows"])), "xs_prepare")
        chk(L.afm_xs_rank_f64(h, Ta, lda, P(an["rows"]), P(an["nrows"]), P(an["skey"]),
                              P(an["sidx"]), P(an["ra"]), P(an["rd"])), "xs_rank")
        chk(L.afm_xs_stats_f64(h, Ta, lda, P(self.an_dates), self.an_nd, P(an["rows"]),
                               P(an["nrows"]), P(an["ra"]), P(an["rd"]), 10, P(an["ic"]),
                               P(an["layer_mean"]), P(an["layer_cnt"]), P(an["port"])),
            "xs_stats")
        chk(L.afm_xs_series_f64(h, self.an_nd, P(an["layer_mean"]), P(an["port"]), P(an["ic"]),
                                P(self.an_year), self.an_nyears, self.an_year0,
                                P(an["cum_layer"]), P(an["ls"]), P(an["cum_port"]), P(an["ir"]),
                                P(an["ir_scratch"])), "xs_series")
        mark("analyzer", 1)

    # ------------------------------------------------------------------------------------------
    def summary(self) -> dict:
        """Host copies of the headline results (after a synchronize)."""
        v = self.pnl["value"].cpu().numpy()
        r = v[1:] / v[:-1] - 1
        out = {"final_value": float(v[-1]), "sharpe": float(r.mean() / r.std(ddof=1)),
               "lasso_beta": self.lasso_beta.cpu().numpy(),
               "lasso_n_iter": int(self.lasso_info[2].item()),
               "lasso_nnz": int((self.lasso_beta[1:] != 0).sum().item()),
               "fm_mean": self.fm_mean.cpu().numpy(), "fm_t": self.fm_t.cpu().numpy(),
               "fm_rank": self.fm_rank.cpu().numpy(), "k": self.reb["k"].cpu().numpy(),
               "status": self.reb["status"].cpu().numpy()}
        if self.cfg.analyzer:
            ic = self.an["ic"].cpu().numpy()
            out["ic_mean"] = np.nanmean(ic, axis=0)
        return out

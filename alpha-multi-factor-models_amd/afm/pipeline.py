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
# a non-reference variant of KKT:433-443 (bench.py's "dense_lasso" line): the 96 factors without
# tmr_ret1d.  With tmr_ret1d in the design the Lasso keeps one coefficient (the headline step
# reads one plane in the predict); without it the fit is dense.
DENSE_FEATURES = tuple(n for n in FEATURES if n != "tmr_ret1d")
# ... and a smaller Lasso penalty (KKT:605 uses 2e-4): on the synthetic panels the 96-column fit
# keeps 1 coefficient at 2e-4 and ~24 at 2e-6 (config-A-sized check with the oracle's CD)
DENSE_ALPHA = 2e-6
N_BLOCKS = 8           # fixed asset blocks of the Gram trees (>= the largest GPU count)
N_CHUNKS = 64          # date chunks of the pooled Gram's row-block partials (2 tree levels)
CHUNK_TREE = (32, 2)   # the chunks of a row-block: groups of 32, then the 2 results

STAGES = ("factors", "zstats", "xs_gram", "lasso", "predict", "rebalance", "pnl", "fm",
          "analyzer")
PIPELINE_STAGES = STAGES
EXCHANGE_STAGES = STAGES + ("exchange",)
# optional step() events around single launches (bench.py's rooflines): the one-pass factor call
# (factor_panel_kernel + masks_kernel) and the pooled Gram's partial kernel (zgram_kernel<7, 1>)
KERNEL_MARKS = ("k_factor", "k_gram")


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
    # the regression design: None = the reference's 97 columns (KKT:433-443, FEATURES).  A stated
    # variant may name another subset -- e.g. DENSE_FEATURES, which drops tmr_ret1d (the
    # undemeaned twin of the target, NT:90-91) so the Lasso keeps many coefficients
    features: tuple | None = None
    # stream placement (moves work between streams only; the outputs are bitwise the same):
    # labels_side -- one GPU: the two label planes on a side stream beside the factor kernel;
    # fm_fork -- one GPU: where the FM per-date Grams fork off the main stream ("gram", "predict",
    # "analyzer" or "rebalance"; measured best: "predict"); main_priority -- the main stream at
    # high priority
    labels_side: bool = True
    fm_fork: str = "predict"
    main_priority: bool = True
    # fm_free_cus -- the FM side stream's kernels avoid this many compute units (a CU-masked
    # stream, afm_stream_create_cu_mask), so the latency-bound tail beside the FM MFMA Grams keeps
    # whole CUs; 0 = an ordinary stream
    fm_free_cus: int = 0
    # fm_grid -- the FM per-date Grams' persistent workgroups (0: one per CU); an A/B knob
    fm_grid: int = 0
    # early_zstats -- the factor panel in two time slabs (afm_factors_range_f64): the train
    # window's z statistics run on a side stream while the second slab builds (a shard's factor
    # kernel leaves most of the GPU free: one wave per job set).  Measured at the N = 8 shard
    # (1,280 assets): 8.97 ms per step either way -- the second slab is the ~17 % of dates after
    # the train window, and the z statistics beside it ran 1.69 instead of 1.03 ms -- so off
    early_zstats: bool = False
    # zstats_slabs -- the factor panel in this many time slabs with the train window's z
    # statistics streamed slab by slab on a side stream right behind them (the recurrences' state
    # carried, afm_zscore_stats_slab_f64): on the smallest grids (the factor launch with one job
    # wave per SIMD, <= 25 blocks: the N = 8 shard) the z statistics then run on the issue slots
    # and CUs the factor kernel leaves free instead of after it.  -1: 6 on those grids, else 0.
    zstats_slabs: int = -1
    # early_fwd -- the analyzer's price rows and forward returns (prediction-independent,
    # KKT:294-296) on a side stream as soon as the all_df rows exist -- one GPU: beside the z
    # statistics; N > 1: after one all-gather of the all_df row words, beside the Grams --
    # instead of at the head of the analyzer stream in the tail
    early_fwd: bool = True
    # reb_split -- N > 1: each rank runs the rebalance of its share of the dates (+ one neighbour
    # per side) and one packed all-gather assembles the books; False: every rank runs every date
    # (the rebalance is latency-bound -- one workgroup per (date, side) -- so a rank's share is
    # not much shorter than all of it) and there is no exchange
    reb_split: bool = True


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


def _round_up(x: int, m: int = 64) -> int:
    return (x + m - 1) // m * m


def _even(n: int, world: int, rank: int):
    return n * rank // world, n * (rank + 1) // world


def _share_rows(ranges, stride: int, device):
    """Rows of the per-rank shares in an all-gathered [world][stride] buffer, in global order
    (rank q's i-th item at row q * stride + i): ONE index_select places every rank's share."""
    import torch
    return torch.as_tensor(np.concatenate([q * stride + np.arange(b - a) for q, (a, b)
                                           in enumerate(ranges)]).astype(np.int64), device=device)


class Pipeline:
    """The chain on one device, or on one rank of ``comm.world`` (``comm``: afm.sharded.Comm).

    Sharding (one process per GPU): rank r owns the asset blocks
    [8r/N, 8(r+1)/N) of the fixed 8-block split -- its factor panel, z-score statistics, pooled
    Gram partials (tree over its row-blocks and blocks) and per-date FM partials.  The
    exchanges: one all-gather of the block results of the pooled Gram (+ the train_end subtree),
    one all-gather of the test-date predictions and row bits, one all_to_all of per-date FM
    partials to the date owners (+ an all-gather of the betas), one all-gather of the rebalance
    results (rebalance dates are split over ranks).  Every sum follows the same fixed trees as
    one device, so every result is bit-identical to N = 1."""

    def __init__(self, grid: PanelGrid, cfg: PipelineConfig | None = None, comm=None):
        import torch
        self.full = grid
        self.comm = comm
        W = comm.world if comm is not None else 1
        rk = comm.rank if comm is not None else 0
        self.W, self.rank = W, rk
        self.cfg = c = cfg or PipelineConfig()
        dev = grid.device
        T, lda, A = grid.T, grid.lda, grid.A
        nch = (T + 63) // 64
        self.T, self.lda, self.A, self.nch = T, lda, A, nch
        self.sp = sp = Split.of(grid.dates, c.train_end, c.valid_end)
        self.features = list(c.features) if c.features is not None else FEATURES
        self.p = p = len(self.features)
        self.p2 = p + 2
        self.pf = len(c.fm_features)
        f64 = dict(dtype=torch.float64, device=dev)
        i64 = dict(dtype=torch.int64, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        L = _lib.lib()
        # ---- asset shard: whole blocks of the fixed split ----
        if N_BLOCKS % W:
            raise ValueError(f"{W} ranks: the GPU count must divide {N_BLOCKS}")
        self.nblk = N_BLOCKS
        self.blk = blk = block_assets(lda)
        self.rb_per_blk = blk // 64
        if self.rb_per_blk > 32:          # afm_gram_tree_f64 merges at most 32 leaves a level
            raise ValueError(f"{A} assets: the pooled-Gram tree holds at most "
                             f"{N_BLOCKS * 32 * 64} assets ({N_BLOCKS} blocks x 32 row-blocks "
                             f"of 64)")
        self.nblk_r = N_BLOCKS // W
        self.ranges = []
        for q in range(W):
            lo = min(q * self.nblk_r * blk, A)
            self.ranges.append((lo, min((q + 1) * self.nblk_r * blk, A)))
        a0, a1 = self.ranges[rk]
        self.a0, self.A_r = a0, a1 - a0
        self.lda_r = lda_r = _round_up(max(self.A_r, 1))
        self.wide = self.nblk_r * blk                  # padded shard width of the exchanges
        if W == 1:
            self.g = grid
        else:
            sl = slice(a0, a0 + lda_r)
            self.g = PanelGrid(dates=grid.dates, ids=grid.ids[a0:a1],
                               close=grid.close[:, sl].contiguous(),
                               volume=grid.volume[:, sl].contiguous(),
                               ret1d=grid.ret1d[:, sl].contiguous(),
                               excess=grid.excess[:, sl].contiguous(),
                               valid=grid.valid[:, sl].contiguous(),
                               vbits=grid.vbits[:, sl].contiguous())
        self.feat = torch.as_tensor(np.array([COL[n] for n in self.features], np.int32),
                                    device=dev)
        # ---- local (shard) buffers ----
        self.out = torch.full((N_FACTORS, T, lda_r), float("nan"), **f64)
        self.nanfree = torch.zeros((nch, lda_r), **i64)
        self.finite = torch.zeros((nch, lda_r), **i64)
        self.alldf = torch.zeros((nch, lda_r), **i64)    # all_df rows (NT:33 dropna)
        self.frows = torch.zeros((nch, lda_r), **i64)    # all_df rows with every feature finite
        self.zrows = torch.zeros((nch, lda_r), **i64)    # rows surviving the z-score dropna
        self.mu = torch.empty((p, lda_r), **f64)
        self.sd = torch.empty((p, lda_r), **f64)
        self.zs = torch.empty((p + 1, lda_r, 2), **f64)
        self.asset_ok = torch.empty(lda_r, **i32)
        self.nrb = (self.A_r + 63) // 64                 # this shard's 64-asset row-blocks
        self.pe = pe = L.afm_zgram_part_bytes(p) // 8
        self.pool_part = torch.empty((max(self.nrb, 1), N_CHUNKS, pe), **f64)
        self.pool_c1 = torch.empty((max(self.nrb, 1) * (N_CHUNKS // CHUNK_TREE[0]), pe), **f64)
        self.pool_rb = torch.empty((max(self.nrb, 1), pe), **f64)
        self.pool_blk = torch.zeros((self.nblk_r + 1, pe), **f64)   # + the train_end subtree
        self.pool_all = torch.zeros((N_BLOCKS, pe), **f64)
        self.te_part = torch.zeros((self.nblk_r, pe), **f64)
        self.te_all = torch.zeros((W, pe), **f64)
        self.pool_g = torch.empty((1, self.p2, self.p2), **f64)
        self.pool_s = torch.zeros((1, self.p2), **f64)   # raw moments: zero shift
        self.te_gram = torch.zeros((1, self.p2, self.p2), **f64)
        self.lasso_beta = torch.empty(p + 1, **f64)
        self.lasso_info = torch.empty(3, **f64)
        # FM design: [1, FM30 factor values, target] per date
        self.fm_cols = torch.as_tensor(np.array([COL[n] for n in c.fm_features], np.int32),
                                       device=dev)
        self.pef = pef = L.afm_zgram_part_bytes(self.pf) // 8
        self.fm_part = torch.zeros((T, self.nblk_r, pef), **f64)
        self.fm_sub = torch.zeros((T, pef), **f64)      # this shard's subtree per date
        self.fdr = [_even(T, W, q) for q in range(W)]   # FM dates owned by each rank
        fd0, fd1 = self.fdr[rk]
        self.fd0, self.fnd = fd0, fd1 - fd0
        self.fnd_max = max(b - a for a, b in self.fdr)
        self.fm_gram = torch.empty((max(self.fnd, 1), self.pf + 2, self.pf + 2), **f64)
        self.fm_shift = torch.zeros((max(self.fnd, 1), self.pf + 2), **f64)
        self.fm_beta_own = torch.full((self.fnd_max, self.pf + 1), float("nan"), **f64)
        self.fm_nobs_own = torch.zeros(self.fnd_max, **f64)
        self.fm_rank_own = torch.zeros(self.fnd_max, **i32)
        if W == 1:
            self.fm_beta, self.fm_nobs, self.fm_rank = (self.fm_beta_own, self.fm_nobs_own,
                                                        self.fm_rank_own)
        else:
            self.fm_beta = torch.empty((T, self.pf + 1), **f64)
            self.fm_nobs = torch.empty(T, **f64)
            self.fm_rank = torch.empty(T, **i32)
        self.fm_mean = torch.empty(self.pf + 1, **f64)
        self.fm_t = torch.empty(self.pf + 1, **f64)
        self.pred_r = torch.full((T, lda_r), float("nan"), **f64)
        # ---- full-width planes the rebalance / analyzer read ----
        if W == 1:
            self.pred, self.zrows_full, self.alldf_full = self.pred_r, self.zrows, self.alldf
            self.target, self.tmr = self.out[TARGET], self.out[TMR]
        else:
            self.pred = torch.full((T, lda), float("nan"), **f64)
            self.zrows_full = torch.zeros((nch, lda), **i64)
            self.alldf_full = torch.zeros((nch, lda), **i64)
            self.target = torch.full((T, lda), float("nan"), **f64)
            self.tmr = torch.full((T, lda), float("nan"), **f64)
            win = c.window if c.window is not None else T
            self.lab0 = 0 if c.window is None else max(0, sp.s0 - int(win) - 1)
        # rebalance dates: the test dates that can carry predictions (a present observation that
        # is not the asset's last -- every other row lacks the target)
        vb = grid.valid.cpu().numpy()
        nxt = np.zeros_like(vb)
        nxt[:-1] = np.flip(np.logical_or.accumulate(np.flip(vb[1:], 0), 0), 0)
        has = (vb & nxt).any(axis=1)
        rd = np.flatnonzero(has[sp.s0:]).astype(np.int32) + sp.s0
        self.nd = nd = len(rd)

        def reb_buffers(n):
            n = max(n, 1)
            return {"k": torch.zeros(n, **i32),
                    "books": torch.full((n, 2, MAX_BOOK), -1, **i32),
                    "weights": torch.zeros((n, 2, MAX_BOOK), **f64),
                    "sums": torch.zeros((n, 4), **f64),
                    "upos": torch.full((n, 2, 2, MAX_BOOK), -1, **i32),
                    "usize": torch.zeros((n, 2), **i64),
                    "status": torch.zeros(n, **i32)}
        self.reb = reb_buffers(nd)
        # rebalance dates of this rank (+ one neighbour per side: the turnover alignment needs the
        # adjacent dates' prediction sets)
        self.reb_split = W > 1 and c.reb_split
        Wr = W if self.reb_split else 1
        self.rrange = [_even(nd, Wr, q) for q in range(Wr)]
        i0, i1 = self.rrange[rk if self.reb_split else 0]
        self.i0, self.i1 = i0, i1
        self.e0, self.e1 = (max(i0 - 1, 0), min(i1 + 1, nd)) if self.reb_split else (0, nd)
        self.rd_ext = torch.from_numpy(rd[self.e0:self.e1].copy()).to(dev)
        self.rdates = torch.from_numpy(rd).to(dev)
        self.reb_ext = reb_buffers(self.e1 - self.e0) if self.reb_split else self.reb
        self.nr_max = max(b - a for a, b in self.rrange)
        self._reb_rows = self._fm_rows = self._an_rows = None
        self._send = {}                     # packed send buffers of the exchanges (N > 1)
        self.pnl = {"value": torch.empty(nd + 1, **f64), "turnover": torch.empty(nd, **f64),
                    "long_ret": torch.empty(nd, **f64), "short_ret": torch.empty(nd, **f64)}
        # analyzer on the test sub-grid (64-date aligned, so the bit words line up)
        self.an_a0 = (sp.s0 // 64) * 64
        Ta = T - self.an_a0
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
            ad = np.arange(sp.s0 - self.an_a0, Ta, dtype=np.int32)   # test dates, sub-grid index
            self.an_dates = torch.from_numpy(ad).to(dev)
            self.an_nd = nad = len(ad)
            # N > 1: each rank evaluates an even share of the test dates (every stage of the
            # analyzer but the final series is per date); one packed all-gather of the per-date
            # results, then every rank runs the series
            self.an_rng = _even(nad, W, rk) if W > 1 else (0, nad)
            self.an_nmax = max(b - a for a, b in (_even(nad, W, q) for q in range(W)))
            years = np.asarray(grid.dates).astype("datetime64[Y]").astype(np.int64) + 1970
            yr = years[self.an_a0 + ad].astype(np.int32)
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
        if c.fm_fork not in ("gram", "predict", "analyzer", "rebalance"):
            raise ValueError(f"fm_fork={c.fm_fork!r}: expected gram, predict, analyzer or "
                             "rebalance")
        self.main = torch.cuda.Stream(device=dev, priority=-8 if c.main_priority else 0)
        self.fm_grid = c.fm_grid          # the FM Grams' persistent grid (0: one per CU)
        if c.fm_free_cus > 0:
            self._side_owner = _lib.cu_mask_stream(dev.index, c.fm_free_cus)
            self.side = self._side_owner.stream
            # one workgroup per CU the masked stream may use: a full-width grid would run the
            # surplus workgroups in a second round
            self.fm_grid = torch.cuda.get_device_properties(dev).multi_processor_count - c.fm_free_cus
        else:
            self.side = torch.cuda.Stream(device=dev, priority=0)
        self.side2 = torch.cuda.Stream(device=dev, priority=0)
        # N > 1: the sequential PnL scan on its own stream, beside the FM exchange / solve and the
        # analyzer's gather + series that follow the rebalance (they no longer wait for it).  One
        # GPU creates no fourth stream: HIP maps streams onto GPU_MAX_HW_QUEUES (4) hardware queues
        # in creation order, and a stream that shares a queue waits behind the other's kernels
        self.side3 = (torch.cuda.Stream(device=dev, priority=-8 if c.main_priority else 0)
                      if W > 1 else self.main)
        self.streams = (self.main, self.side, self.side2) + ((self.side3,) if W > 1 else ())
        self.labels_done = torch.cuda.Event()
        self.fwd_early = False
        # early z statistics: the first slab ends at the first 64-date boundary past the train
        # window (the slab API's alignment)
        self.ta = min(((sp.tr1 + 63) // 64) * 64, T)
        nslab = c.zstats_slabs
        if nslab < 0:
            ncu = torch.cuda.get_device_properties(dev).multi_processor_count
            nslab = 6 if ((self.A_r + 63) // 64) * 10 <= ncu else 0
        self.stream_z = nslab >= 2 and self.A_r > 0 and sp.tr1 > 0 and T >= 128
        if self.stream_z:
            bounds = sorted({0, T} | {min(T, ((i * T // nslab + 63) // 64) * 64)
                                      for i in range(1, nslab)})
            self.zbounds = bounds
            self.zstate = torch.empty((5, p, lda_r), **f64)
            self.zparts = [torch.empty(int(L.afm_factors_part_words(self.ctx.handle, self.A_r,
                                                                    lda_r, a, z)), **i64)
                           for a, z in zip(bounds[:-1], bounds[1:])]
            self.zslab_done = [torch.cuda.Event() for _ in bounds[:-1]]
            self.zstats_done = torch.cuda.Event()
        self.early = (bool(c.early_zstats) and not self.stream_z and self.A_r > 0 and self.ta < T)
        if self.early or self.stream_z:
            nb = int(L.afm_factors_state_bytes(self.ctx.handle, self.A_r))
            self.fstate = torch.empty(nb // 8 + 1, **f64)
            self.slab1_done = torch.cuda.Event()
            if not self.stream_z:
                self.zstats_done = torch.cuda.Event()

    @property
    def labels_in_factor_stage(self) -> bool:
        """The two label planes are written inside the ``factors`` stage (main stream) rather
        than on a side stream beside it: one GPU with ``labels_side`` off (bench.py's roofline
        counts their bytes against that stage only then)."""
        return self.W == 1 and not self.cfg.labels_side

    def n_asset_days_local(self) -> int:
        return int(self.g.valid.sum().item())

    # ------------------------------------------------------------------------------------------
    def _pooled_blocks(self, h, t0, nt, mark=None):
        """This shard's pooled-Gram block results (rows of the dates [t0, t0 + nt)): row-block x
        chunk partials, then the tree -- the chunks of a row-block (32, then 2), the row-blocks
        of an asset block -> pool_blk[0:nblk_r]."""
        L, P, chk = _lib.lib(), _lib.ptr, _lib.check
        T, lda, p = self.T, self.lda_r, self.p
        self.pool_blk.zero_()
        if self.nrb == 0:
            return
        if mark is not None:
            mark("k_gram", 0)
        chk(L.afm_zpool_f64(h, P(self.out), T * lda, lda, P(self.feat), None, p, TARGET,
                            P(self.zs), p, P(self.zrows), t0, nt, 0, self.nrb, self.A_r,
                            N_CHUNKS, P(self.pool_part), 0), "zpool")
        if mark is not None:
            mark("k_gram", 1)
        c1, c2 = CHUNK_TREE
        chk(L.afm_gram_tree_f64(h, p, P(self.pool_part), self.nrb * N_CHUNKS, c1, 0,
                                P(self.pool_c1)), "tree chunks")
        chk(L.afm_gram_tree_f64(h, p, P(self.pool_c1), self.nrb * c2, c2, 0, P(self.pool_rb)),
            "tree chunks 2")
        chk(L.afm_gram_tree_f64(h, p, P(self.pool_rb), self.nrb, self.rb_per_blk, 0,
                                P(self.pool_blk)), "tree row-blocks")

    def _te_subtree(self, h, t):
        """This shard's subtree of the train_end date's Gram -> pool_blk[nblk_r]."""
        L, P, chk = _lib.lib(), _lib.ptr, _lib.check
        T, lda, p = self.T, self.lda_r, self.p
        if self.nrb == 0:
            return
        chk(L.afm_zgram_f64(h, P(self.out), T * lda, lda, P(self.feat), None, p, TARGET,
                            P(self.zs), p, P(self.zrows), t, 1, self.nblk_r, 0, self.blk,
                            self.A_r, P(self.te_part), 0), "zgram date")
        chk(L.afm_gram_tree_f64(h, p, P(self.te_part), self.nblk_r, self.nblk_r, 0,
                                P(self.pool_blk[self.nblk_r:])), "tree date")

    def _fm_local(self, h):
        """This shard's per-date FM30 partials over the z-score rows, merged over its blocks ->
        fm_sub [T]."""
        L, P, chk = _lib.lib(), _lib.ptr, _lib.check
        T, lda, pf = self.T, self.lda_r, self.pf
        if self.nrb == 0:
            return
        chk(L.afm_zgram_f64(h, P(self.out), T * lda, lda, P(self.fm_cols), None, pf, TARGET,
                            None, 0, P(self.zrows), 0, T, self.nblk_r, 0, self.blk, self.A_r,
                            P(self.fm_part), self.fm_grid), "zgram fm")
        chk(L.afm_gram_tree_f64(h, pf, P(self.fm_part), T * self.nblk_r, self.nblk_r, 0,
                                P(self.fm_sub)), "tree fm blocks")

    def _fm_solve(self, h, sub):
        """Owned dates: the rank subtrees ``sub`` [fnd][W][part] -> Grams, solves; every rank then
        gets every date's betas and the FM statistics."""
        L, P, chk = _lib.lib(), _lib.ptr, _lib.check
        c, pf, T = self.cfg, self.pf, self.T
        if self.fnd > 0:
            chk(L.afm_gram_tree_f64(h, pf, P(sub), self.fnd * self.W, self.W, 1,
                                    P(self.fm_gram)), "tree fm ranks")
            chk(L.afm_ols_solve_f64(h, P(self.fm_gram), P(self.fm_shift), pf, self.fnd, c.tol,
                                    P(self.fm_beta_own), P(self.fm_nobs_own),
                                    P(self.fm_rank_own)), "fm solve")

    def _factors_streamed(self, h, lab_side, mark):
        """The factor panel in time slabs (zbounds) on the main stream, each slab's all_df rows
        right behind it, and the train window's z statistics streamed slab by slab on the side
        stream as each slab lands (afm_zscore_stats_slab_f64, every (feature, asset) recurrence
        carried): bitwise the panel, statistics and row sets of one call each.  The label planes
        go first, once, on the second side stream (inputs only; tmr_ret1d is a feature) -- not
        inside every factor slab; with ``labels_side`` off, on the main stream ahead of the first
        slab, inside the factors stage)."""
        import torch
        L, P, chk = _lib.lib(), _lib.ptr, _lib.check
        g, sp, T, lda_r, p, A_r = self.g, self.sp, self.T, self.lda_r, self.p, self.A_r
        lab_stream = self.side2 if lab_side else self.main
        with torch.cuda.stream(lab_stream):
            h2 = self.ctx.bind_stream()
            chk(L.afm_labels_f64(h2, T, lda_r, 0, T, P(g.excess), P(g.ret1d), P(g.vbits),
                                 P(self.out[TARGET]), P(self.out[TMR])), "labels")
            self.labels_done.record(lab_stream)
        h = self.ctx.bind_stream()
        b, tr1 = self.zbounds, sp.tr1
        for i in range(len(b) - 1):
            t0, t1 = b[i], b[i + 1]
            # the slab on the main stream; its row masks, all_df rows and z statistics on the side
            # stream beside the next slab (the next slab needs only the carried factor state)
            need = int(L.afm_factors_part_words(self.ctx.handle, A_r, lda_r, t0, t1))
            if need > self.zparts[i].numel():    # (an execution option changed the launch shape)
                self.zparts[i] = torch.empty(need, dtype=torch.int64, device=self.out.device)
            part = self.zparts[i]
            chk(L.afm_factors_range_part_f64(h, T, A_r, lda_r, t0, t1, P(g.close), P(g.volume),
                                             P(g.vbits), P(self.out), P(self.fstate), P(part)),
                "factors slab")
            self.zslab_done[i].record(self.main)
            with torch.cuda.stream(self.side):
                hs = self.ctx.bind_stream()
                self.side.wait_event(self.zslab_done[i])
                chk(L.afm_factor_masks_f64(hs, T, A_r, lda_r, t0, t1, P(g.vbits), P(part),
                                           P(self.nanfree), P(self.finite)), "factor masks")
                for src, dst in ((self.nanfree, self.alldf), (self.finite, self.frows)):
                    chk(L.afm_drop_last_obs_bits_range(hs, T, lda_r, P(g.vbits), P(src), P(dst),
                                                       t0, t1), "last-obs rows")
                if t0 < tr1:
                    if i == 0:
                        self.side.wait_event(self.labels_done)
                        mark("zstats", 0)
                    last = t1 >= tr1
                    chk(L.afm_zscore_stats_slab_f64(hs, P(self.out), T * lda_r, T, lda_r,
                                                    P(self.feat), p, P(self.alldf), t0,
                                                    min(t1, tr1), P(self.zstate), int(i == 0),
                                                    int(last), P(self.mu), P(self.sd)),
                        "zscore stats slab")
                    if last:
                        chk(L.afm_zstats_finalize_f64(hs, P(self.mu), P(self.sd), p, lda_r,
                                                      P(self.zs), P(self.asset_ok)),
                            "zstats finalize")
                        mark("zstats", 1)
            h = self.ctx.bind_stream()
        mark("factors", 1)
        self.zstats_done.record(self.side)        # every slab's masks, rows and statistics
        self.main.wait_event(self.zstats_done)
        chk(L.afm_row_bits(h, self.nch, lda_r, P(self.frows), None, P(self.asset_ok), 0, T,
                           P(self.zrows)), "z rows")

    def _factors_early(self, h, lab_side, mark):
        """The factor panel in two slabs [0, ta) and [ta, T) on the main stream; the train
        window's z statistics (and the z-score row bits of the first slab) on the side stream
        beside the second slab.  Bitwise the same panel, statistics and row sets as one call."""
        import torch
        L, P, chk = _lib.lib(), _lib.ptr, _lib.check
        g, sp, T, lda_r, p, ta = self.g, self.sp, self.T, self.lda_r, self.p, self.ta
        A_r, wa = self.A_r, self.ta // 64
        lab = (None, None) if lab_side else (P(g.ret1d), P(g.excess))
        chk(L.afm_factors_range_f64(h, T, A_r, lda_r, 0, ta, P(g.close), P(g.volume), *lab,
                                    P(g.vbits), P(self.out), P(self.nanfree), P(self.finite),
                                    P(self.fstate)), "factors slab 1")
        if lab_side:
            with torch.cuda.stream(self.side2):
                h2 = self.ctx.bind_stream()
                chk(L.afm_labels_f64(h2, T, lda_r, 0, T, P(g.excess), P(g.ret1d), P(g.vbits),
                                     P(self.out[TARGET]), P(self.out[TMR])), "labels")
                self.labels_done.record(self.side2)
            h = self.ctx.bind_stream()
        for src, dst in ((self.nanfree, self.alldf), (self.finite, self.frows)):
            chk(L.afm_drop_last_obs_bits_range(h, T, lda_r, P(g.vbits), P(src), P(dst), 0, ta),
                "last-obs rows 1")
        self.slab1_done.record(self.main)
        with torch.cuda.stream(self.side):
            hs = self.ctx.bind_stream()
            self.side.wait_event(self.slab1_done)
            if lab_side:
                self.side.wait_event(self.labels_done)          # tmr_ret1d is a feature
            mark("zstats", 0)
            chk(L.afm_zscore_stats_f64(hs, P(self.out), T * lda_r, T, lda_r, P(self.feat), p,
                                       P(self.alldf), 0, sp.tr1, P(self.mu), P(self.sd)),
                "zscore stats")
            chk(L.afm_zstats_finalize_f64(hs, P(self.mu), P(self.sd), p, lda_r, P(self.zs),
                                          P(self.asset_ok)), "zstats finalize")
            chk(L.afm_row_bits(hs, wa, lda_r, P(self.frows), None, P(self.asset_ok), 0, ta,
                               P(self.zrows)), "z rows 1")
            mark("zstats", 1)
            self.zstats_done.record(self.side)
        h = self.ctx.bind_stream()
        chk(L.afm_factors_range_f64(h, T, A_r, lda_r, ta, T, P(g.close), P(g.volume), *lab,
                                    P(g.vbits), P(self.out), P(self.nanfree), P(self.finite),
                                    P(self.fstate)), "factors slab 2")
        for src, dst in ((self.nanfree, self.alldf), (self.finite, self.frows)):
            chk(L.afm_drop_last_obs_bits_range(h, T, lda_r, P(g.vbits), P(src), P(dst), ta, T),
                "last-obs rows 2")
        mark("factors", 1)
        self.main.wait_event(self.zstats_done)
        chk(L.afm_row_bits(h, self.nch - wa, lda_r, P(self.frows[wa:]), None, P(self.asset_ok),
                           0, T - ta, P(self.zrows[wa:])), "z rows 2")

    def step(self, events: dict | None = None):
        """One pass of the chain.  ``events``: optional {stage: (start, end)} CUDA events."""
        import torch
        L, P, chk = _lib.lib(), _lib.ptr, _lib.check
        g, c, sp, cm = self.g, self.cfg, self.sp, self.comm
        T, lda_r, p, W, nch = self.T, self.lda_r, self.p, self.W, self.nch
        full = self.full
        caller = torch.cuda.current_stream(full.device)
        for s in self.streams:
            s.wait_stream(caller)

        def mark(stage, which):
            if events is not None and stage in events:
                events[stage][which].record()

        with torch.cuda.stream(self.main):
            h = self.ctx.bind_stream()
            mark("factors", 0)
            # one GPU: the two label planes on the side stream, enqueued after the factor kernel
            # (it runs on the CUs the factor workgroups leave free); zstats waits for them
            lab_side = W == 1 and c.labels_side
            if self.stream_z:
                self._factors_streamed(h, lab_side, mark)
                h = self.ctx.bind_stream()
            elif self.early:
                self._factors_early(h, lab_side, mark)
                h = self.ctx.bind_stream()
            elif self.A_r > 0:
                mark("k_factor", 0)
                chk(L.afm_factors_f64(h, T, self.A_r, lda_r, P(g.close), P(g.volume),
                                      None if lab_side else P(g.ret1d),
                                      None if lab_side else P(g.excess), P(g.vbits), P(self.out),
                                      P(self.nanfree), P(self.finite)), "factors")
                mark("k_factor", 1)
                if lab_side:
                    with torch.cuda.stream(self.side2):
                        h2 = self.ctx.bind_stream()
                        chk(L.afm_labels_f64(h2, T, lda_r, 0, T, P(g.excess), P(g.ret1d),
                                             P(g.vbits), P(self.out[TARGET]), P(self.out[TMR])),
                            "labels")
                        self.labels_done.record(self.side2)
                    h = self.ctx.bind_stream()
                chk(L.afm_drop_last_obs_bits(h, T, lda_r, P(g.vbits), P(self.nanfree),
                                             P(self.alldf)), "all_df rows")
                chk(L.afm_drop_last_obs_bits(h, T, lda_r, P(g.vbits), P(self.finite),
                                             P(self.frows)), "finite rows")
            one_pass = not (self.early or self.stream_z)
            if one_pass:
                mark("factors", 1)
            self.fwd_early = c.analyzer and c.early_fwd
            if self.fwd_early and W == 1:
                self.side2.wait_stream(self.main)                # the all_df rows
                with torch.cuda.stream(self.side2):
                    self._analyzer_fwd()
                h = self.ctx.bind_stream()
            if one_pass:
                mark("zstats", 0)
            if self.A_r > 0 and one_pass:
                if lab_side:
                    self.main.wait_event(self.labels_done)          # tmr_ret1d is a feature
                chk(L.afm_zscore_stats_f64(h, P(self.out), T * lda_r, T, lda_r, P(self.feat), p,
                                           P(self.alldf), 0, sp.tr1, P(self.mu), P(self.sd)),
                    "zscore stats")
                chk(L.afm_zstats_finalize_f64(h, P(self.mu), P(self.sd), p, lda_r, P(self.zs),
                                              P(self.asset_ok)), "zstats finalize")
                chk(L.afm_row_bits(h, nch, lda_r, P(self.frows), None, P(self.asset_ok), 0, T,
                                   P(self.zrows)), "z rows")
            if one_pass:
                mark("zstats", 1)
            if W > 1:           # full-width label planes for the rebalance, during the Grams
                with torch.cuda.stream(self.side2):
                    h2 = self.ctx.bind_stream()
                    chk(L.afm_labels_f64(h2, T, full.lda, self.lab0, T, P(full.excess),
                                         P(full.ret1d), P(full.vbits), P(self.target),
                                         P(self.tmr)), "labels")
                    self.labels_done.record(self.side2)
                if self.fwd_early:
                    # the analyzer's price rows and forward returns need the whole cross-section's
                    # all_df rows only (not the predictions): gathered now, beside the Grams, so
                    # the analyzer's prediction-dependent chain starts right at the predict
                    self.side2.wait_stream(self.main)            # the all_df rows (after zstats)
                    with torch.cuda.stream(self.side2):
                        self._gather_alldf()
                        self._analyzer_fwd()
                h = self.ctx.bind_stream()
            mark("xs_gram", 0)
            self._pooled_blocks(h, 0, sp.v1, mark)                  # train + valid rows
            if sp.dup:                                              # train_end counted twice
                self._te_subtree(h, sp.tr1 - 1)
            if W > 1:
                mark("exchange", 0)
                gb = cm.all_gather(self.pool_blk)                   # [W][nblk_r + 1][part]
                self.pool_all.copy_(gb[:, :self.nblk_r].reshape(N_BLOCKS, self.pe))
                self.te_all.copy_(gb[:, self.nblk_r])
                mark("exchange", 1)
                h = self.ctx.bind_stream()
                blocks, te_leaves, nte = self.pool_all, self.te_all, W
            else:
                blocks, te_leaves, nte = self.pool_blk, self.pool_blk[self.nblk_r:], 1
            chk(L.afm_gram_tree_f64(h, p, P(blocks), N_BLOCKS, N_BLOCKS, 1, P(self.pool_g)),
                "tree blocks")
            if sp.dup:
                chk(L.afm_gram_tree_f64(h, p, P(te_leaves), nte, nte, 1, P(self.te_gram)),
                    "tree train_end")
                chk(L.afm_vec_add_f64(h, self.p2 * self.p2, P(self.te_gram), P(self.pool_g)),
                    "dup")
            mark("xs_gram", 1)
            # side stream: this shard's per-date FM30 partials (nothing downstream reads them),
            # forked after the pooled Gram -- run beside it, both MFMA kernels slow down (A/B on
            # MI355X: pooled Gram 12.7 ms alone, 23 ms beside the FM Grams).  One GPU: forked
            # after the predict, ahead of the analyzer (A/B over 5 runs: 35.29 vs 35.40 ms/step
            # forked after the Gram; 36.4-37.0 after the analyzer, 36.5-36.7 after the
            # rebalance).  AFM_FM_FORK=gram|predict|analyzer|rebalance: A/B.
            def fork_fm():
                self.side.wait_stream(self.main)
                with torch.cuda.stream(self.side):
                    hs = self.ctx.bind_stream()
                    mark("fm", 0)
                    self._fm_local(hs)
                    if W == 1:
                        self._fm_solve(hs, self.fm_sub)
                        self._fm_stats(hs)
                    mark("fm", 1)
                return self.ctx.bind_stream()

            fm_at = c.fm_fork if W == 1 else "gram"
            if fm_at == "gram":
                h = fork_fm()
            mark("lasso", 0)
            chk(L.afm_lasso_fit_f64(h, P(self.pool_g), P(self.pool_s), p, c.alpha, c.max_iter,
                                    c.lasso_tol, 0, P(self.lasso_beta), P(self.lasso_info)),
                "lasso")
            mark("lasso", 1)
            mark("predict", 0)
            if self.A_r > 0:
                chk(L.afm_zpredict_f64(h, P(self.out), T * lda_r, lda_r, sp.s0, T - sp.s0,
                                       P(self.feat), p, P(self.zs), P(self.lasso_beta),
                                       P(self.zrows), P(self.pred_r)), "predict")
            if W > 1:                          # the whole cross-section of the test dates
                self._gather_test_planes()
                h = self.ctx.bind_stream()
            mark("predict", 1)
            if fm_at == "predict":
                h = fork_fm()
            if c.analyzer:
                self.side2.wait_stream(self.main)
                with torch.cuda.stream(self.side2):
                    self._analyzer(mark)
                h = self.ctx.bind_stream()
            if fm_at == "analyzer":
                h = fork_fm()
            mark("rebalance", 0)
            if W > 1:
                self.main.wait_event(self.labels_done)     # the label planes
            x = self.reb_ext
            ne = self.e1 - self.e0
            if ne > 0:
                chk(L.afm_rebalance_f64(h, T, full.A, full.lda, P(self.rd_ext), ne, P(self.pred),
                                        P(full.tbits), P(self.target), P(self.zrows_full), 0,
                                        sp.tr1, -1 if c.window is None else int(c.window),
                                        P(full.close), P(self.tmr), c.top_n, c.lo, c.hi,
                                        P(x["k"]), P(x["books"]), P(x["weights"]), P(x["sums"]),
                                        P(x["upos"]), P(x["usize"]), P(x["status"])), "rebalance")
            if self.reb_split:
                self._gather_rebalance()
                h = self.ctx.bind_stream()
            mark("rebalance", 1)
            if fm_at == "rebalance":
                h = fork_fm()
            r, q = self.reb, self.pnl

            def pnl_scan(hh):
                mark("pnl", 0)
                chk(L.afm_pnl_scan_f64(hh, self.nd, P(r["k"]), P(r["books"]), P(r["sums"]),
                                       P(r["upos"]), P(r["usize"]), c.v0, c.rate, P(q["value"]),
                                       P(q["turnover"]), P(q["long_ret"]), P(q["short_ret"])),
                    "pnl")
                mark("pnl", 1)
            if W == 1:
                pnl_scan(h)
            else:
                # the scan on its own stream; the FM exchange (per-date subtrees -> date owners,
                # solves, betas) and the analyzer's gather + series run beside it on the main and
                # second side streams, issued in this order on every rank (RCCL runs a group's
                # collectives in issue order)
                self.side3.wait_stream(self.main)
                with torch.cuda.stream(self.side3):
                    pnl_scan(self.ctx.bind_stream())
                h = self.ctx.bind_stream()
                self.main.wait_stream(self.side)
                self._fm_exchange()
                if c.analyzer:
                    with torch.cuda.stream(self.side2):
                        self._analyzer_series(mark)
        for s in self.streams:
            caller.wait_stream(s)
        self.ctx.bind_stream()

    # ---- exchanges (N > 1) -------------------------------------------------------------------
    def _send_buffer(self, key, specs, device):
        """The persistent packed send buffer of one exchange (made on its first step)."""
        from .packing import SendBuffer
        sb = self._send.get(key)
        if sb is None:
            sb = self._send[key] = SendBuffer(specs, device)
        return sb

    def _gather_analyzer(self):
        """The per-date analyzer results of every rank's date share -> the full arrays (one
        packed all-gather, shares padded to the largest)."""
        import torch
        an, (j0, j1), n = self.an, self.an_rng, self.an_nmax
        keys = ("ic", "layer_mean", "layer_cnt", "port")
        sb = self._send_buffer("an", [((n,) + tuple(an[k].shape[1:]), an[k].dtype, 0)
                                      for k in keys], an["ic"].device)
        for k, part in zip(keys, sb.parts):          # rows past the share stay zero
            part[:j1 - j0].copy_(an[k][j0:j1])
        got = self.comm.all_gather_buffer(sb)
        if self._an_rows is None:           # gathered row (rank q, j) of every analyzer date
            self._an_rows = _share_rows([_even(self.an_nd, self.W, q) for q in range(self.W)], n,
                                        an["ic"].device)
        for k, g in zip(keys, got):         # one gather per key, not one copy per rank
            torch.index_select(g.reshape((-1,) + tuple(g.shape[2:])), 0, self._an_rows,
                               out=an[k][:self.an_nd])

    def _place(self, dst, gathered, rows=None):
        """Scatter per-rank shard columns ([W][rows][wide]) into a full-width plane.  Rank q's
        columns start at q * wide (the fixed block split), so the ranks side by side ARE the
        plane's first W * wide columns: the full-width ranks in ONE strided copy straight into the
        plane (no reordered intermediate), the last (short) rank in a second -- not one copy per
        rank (each small copy is a launch the step waits on).  Columns from A on are untouched."""
        A = self.ranges[-1][1]
        if A == 0:
            return
        W, nr, wide = gathered.shape[0], gathered.shape[1], gathered.shape[2]
        d = dst if rows is None else dst[rows]
        k = (W - 1) * wide                  # the full-width ranks' columns
        if k <= A and A - k <= wide:
            if W > 1:
                d[:, :k].view(nr, W - 1, wide).copy_(gathered[:W - 1].permute(1, 0, 2))
            d[:, k:A] = gathered[W - 1, :, :A - k]
            return
        side = gathered.permute(1, 0, 2).reshape(nr, W * wide)
        d[:, :A] = side[:, :A]

    def _gather_test_planes(self):
        """The test dates' predictions and the z-score / all_df row words of every rank's asset
        shard -> the full-width planes (one packed all-gather; the all_df words already went
        out with the forward returns when those run early, ``_gather_alldf``)."""
        import torch
        s0, wide, A_r = self.sp.s0, self.wide, self.A_r
        specs = [((self.T - s0, wide), torch.float64, float("nan")),
                 ((self.nch, wide), torch.int64, 0)]
        with_alldf = not self.fwd_early
        if with_alldf:
            specs.append(((self.nch, wide), torch.int64, 0))
        sb = self._send_buffer("test" if with_alldf else "test_noad", specs, self.pred_r.device)
        pr, zb = sb.parts[:2]                       # columns past A_r keep NaN / 0
        if A_r > 0:
            pr[:, :A_r].copy_(self.pred_r[s0:, :A_r])
            zb[:, :A_r].copy_(self.zrows[:, :A_r])
            if with_alldf:
                sb.parts[2][:, :A_r].copy_(self.alldf[:, :A_r])
        got = self.comm.all_gather_buffer(sb)
        self._place(self.pred, got[0], rows=slice(s0, self.T))
        self._place(self.zrows_full, got[1])
        if with_alldf:
            self._place(self.alldf_full, got[2])

    def _gather_alldf(self):
        """Every rank's all_df row words -> the full-width ``alldf_full`` (one all-gather)."""
        import torch
        sb = self._send_buffer("alldf", [((self.nch, self.wide), torch.int64, 0)],
                               self.alldf.device)
        if self.A_r > 0:
            sb.parts[0][:, :self.A_r].copy_(self.alldf[:, :self.A_r])
        self._place(self.alldf_full, self.comm.all_gather_buffer(sb)[0])

    def _gather_rebalance(self):
        import torch
        x = self.reb_ext
        lo = self.i0 - self.e0
        n_own = self.i1 - self.i0
        sb = self._send_buffer("reb", [((self.nr_max,) + tuple(v.shape[1:]), v.dtype, 0)
                                       for v in x.values()], x["k"].device)
        for v, part in zip(x.values(), sb.parts):    # rows past the share stay zero
            part[:n_own].copy_(v[lo:lo + n_own])
        if self._reb_rows is None:          # gathered row (rank q, i) of every rebalance date
            self._reb_rows = _share_rows(self.rrange, self.nr_max, x["k"].device)
        for k, gath in zip(x.keys(), self.comm.all_gather_buffer(sb)):
            if self.nd > 0:                 # one gather per key, not one copy per rank
                torch.index_select(gath.reshape((-1,) + tuple(gath.shape[2:])), 0,
                                   self._reb_rows, out=self.reb[k][:self.nd])

    def _fm_exchange(self):
        import torch
        W, pef = self.W, self.pef
        splits = [b - a for a, b in self.fdr]
        recv = self.comm.all_to_all(self.fm_sub, splits, [self.fnd] * W)   # [W * fnd][part]
        sub = recv.view(W, self.fnd, pef).transpose(0, 1).contiguous()     # [fnd][W][part]
        h = self.ctx.bind_stream()
        self._fm_solve(h, sub)
        got = self.comm.all_gather_packed([self.fm_beta_own, self.fm_nobs_own, self.fm_rank_own])
        if self._fm_rows is None:           # gathered row (rank q, i) of every FM date
            self._fm_rows = _share_rows(self.fdr, self.fnd_max, self.fm_beta.device)
        for g, dst in zip(got, (self.fm_beta, self.fm_nobs, self.fm_rank)):
            torch.index_select(g.reshape((-1,) + tuple(g.shape[2:])), 0, self._fm_rows, out=dst)
        self._fm_stats(self.ctx.bind_stream())

    def _fm_stats(self, h):
        L, P, chk = _lib.lib(), _lib.ptr, _lib.check
        chk(L.afm_fama_macbeth_f64(h, P(self.fm_beta), P(self.fm_rank), self.T, self.pf + 1,
                                   P(self.fm_mean), P(self.fm_t)), "fama_macbeth")

    # ------------------------------------------------------------------------------------------
    def _analyzer(self, mark):
        """AlphaSignalAnalyzer(lasso_predict, price_data=df_test[['close_price']]).run()
        (KKT:630-631) on the test sub-grid, no host synchronisation."""
        L, P, chk = _lib.lib(), _lib.ptr, _lib.check
        full, sp, an = self.full, self.sp, self.an
        lda, a0, Ta = full.lda, self.an_a0, self.Ta
        h = self.ctx.bind_stream()
        mark("analyzer", 0)
        if not self.fwd_early:
            self._analyzer_fwd()
        j0, j1 = self.an_rng
        d0 = sp.s0 - a0 + j0                        # sub-grid dates [d0, d1) of this rank
        d1 = d0 + (j1 - j0)
        if j1 > j0:
            chk(L.afm_xs_prepare_range_f64(h, Ta, full.A, lda, d0, d1, P(self.pred[a0:]),
                                           P(an["fr"]), P(an["scratch"]), P(an["rows"]),
                                           P(an["rows_idx"]), P(an["nrows"])), "xs_prepare")
            chk(L.afm_xs_layers_f64(h, d1 - d0, lda, P(an["rows"][0, d0:]), P(an["nrows"][d0:]),
                                    P(an["skey"][d0:]), P(an["sidx"][d0:]), P(an["ra"][d0:]),
                                    P(an["rd"][d0:])), "xs_layers")
            chk(L.afm_xs_stats_f64(h, Ta, lda, P(self.an_dates[j0:]), j1 - j0, P(an["rows"]),
                                   P(an["nrows"]), P(an["ra"]), P(an["rd"]), 10, P(an["ic"][j0:]),
                                   P(an["layer_mean"][j0:]), P(an["layer_cnt"][j0:]),
                                   P(an["port"][j0:])), "xs_stats")
        if self.W > 1:
            return          # the all-gather and the series follow the main chain's exchanges
        self._analyzer_series(mark)

    def _analyzer_fwd(self):
        """The analyzer's df_test price rows and forward returns (KKT:294-296): they read the close
        plane and the all_df rows only, not the predictions."""
        L, P, chk = _lib.lib(), _lib.ptr, _lib.check
        full, sp, an, a0 = self.full, self.sp, self.an, self.an_a0
        h = self.ctx.bind_stream()
        chk(L.afm_row_bits(h, self.nch, full.lda, P(self.alldf_full), None, None, sp.s0, self.T,
                           P(self.price_bits)), "price rows")
        cb = a0 // 64
        chk(L.afm_fwd_returns_f64(h, self.Ta, full.lda, P(full.close[a0:]),
                                  P(self.price_bits[cb:]), P(an["fr"])), "fwd_returns")

    def _analyzer_series(self, mark):
        L, P, chk = _lib.lib(), _lib.ptr, _lib.check
        an = self.an
        if self.W > 1:
            self._gather_analyzer()
        h = self.ctx.bind_stream()
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

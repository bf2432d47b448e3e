"""Seeded synthetic OHLCV panels (SURVEY.md §8(d) "Synthetic inputs").

The reference's data files (``data_set_N.csv``, ``security_reference_data_w_ret1d_*.csv``;
schema at ``KKT Yuliang Jiang.py:45-56,85,138,150-161``) are not shipped, so every test, golden
vector and benchmark runs on this generator:

* log-price random walk, mu=3e-4, sigma=0.02, start 50
* volume ~ round(lognormal(13, 0.5))
* ``ret1d`` = close ratio - 1 (the underlying walk, so a hole day still moves the price)
* ``excess_ret1d`` = ret1d - per-date mean over the rows present that day (``KKT:158-161``,
  including its ``ret1d <= 1`` filter)
* ``in_trading_universe`` = 'Y' with probability ``tradable_p``
* listing offsets uniform in [0, T*listing_frac), plus ``hole_frac`` missing asset-days

A panel is held in the *calendar grid* layout the GPU path uses: ``[T][lda]`` row-major arrays
(date-major, asset-minor, ``lda`` = A rounded up to 64) with a validity mask.  ``to_frame``
turns it into the reference's long DataFrame (one row per present asset-day).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

LANES = 64


def round_up(x: int, m: int = LANES) -> int:
    return (x + m - 1) // m * m


@dataclass
class Panel:
    dates: np.ndarray          # [T] datetime64[ns]
    ids: np.ndarray            # [A] int64 security ids (ascending)
    close: np.ndarray          # [T][lda] float64
    volume: np.ndarray         # [T][lda]
    ret1d: np.ndarray          # [T][lda]
    excess: np.ndarray         # [T][lda]
    valid: np.ndarray          # [T][lda] bool  (asset-day present in the long panel)
    tradable: np.ndarray       # [T][lda] bool  (in_trading_universe == 'Y')
    group_id: np.ndarray = field(default=None)  # [A] int64

    @property
    def T(self) -> int:
        return self.close.shape[0]

    @property
    def A(self) -> int:
        return len(self.ids)

    @property
    def lda(self) -> int:
        return self.close.shape[1]

    @property
    def n_asset_days(self) -> int:
        return int(self.valid.sum())


def make_panel(n_assets: int, n_days: int, seed: int = 2023, *, hole_frac: float = 0.002,
               listing_frac: float = 0.1, tradable_p: float = 1.0, start: str = "2000-01-03",
               edge_cases: bool = False, min_obs: int = 0) -> Panel:
    """Generate a ragged, holey panel.  ``edge_cases`` plants the traps the reference's
    semantics hinge on (constant-price runs, zero-volume days, a short-lived asset)."""
    rng = np.random.default_rng(seed)
    T, A = int(n_days), int(n_assets)
    lda = round_up(max(A, 1))
    dates = np.asarray(np.busday_offset(np.datetime64(start, "D"), np.arange(T), roll="forward"),
                       dtype="datetime64[ns]")
    ids = (1000 + 7 * np.arange(A)).astype(np.int64)

    eps = rng.normal(3e-4, 0.02, size=(T + 1, A))
    logp = np.log(50.0) + np.cumsum(eps, axis=0)
    px = np.exp(logp)                       # px[0] is the pre-sample close
    close = px[1:]
    volume = np.round(rng.lognormal(13.0, 0.5, size=(T, A)))

    listing = rng.integers(0, max(1, int(T * listing_frac)), size=A)
    if min_obs:
        listing = np.minimum(listing, max(0, T - min_obs))
    valid = np.arange(T)[:, None] >= listing[None, :]
    holes = rng.random((T, A)) < hole_frac
    valid &= ~holes

    if edge_cases and A >= 4 and T >= 120:
        # constant-price run (zero-variance windows -> 0/0 corr, same-value rolling rule)
        a = 1
        t0 = max(listing[a], 0) + 70
        close[t0:t0 + 25, a] = close[t0, a]
        # zero-volume day (vol_change -> inf, then -1) and a two-day zero run (0/0 -> NaN)
        a = 2
        t1 = max(listing[a], 0) + 80
        volume[t1, a] = 0.0
        volume[t1 + 30:t1 + 32, a] = 0.0
        # a short-lived asset: fewer than the 58 observations the warm-up needs
        a = 3
        valid[:, a] = False
        valid[T // 2:T // 2 + 40, a] = True
        # exactly equal consecutive closes (OBV treats diff == 0 as down)
        a = 0
        t2 = max(listing[a], 0) + 90
        close[t2 + 1, a] = close[t2, a]

    prev = np.vstack([px[:1], close[:-1]])
    ret1d = close / prev - 1.0

    # excess_ret1d: per-date demean over present rows with ret1d <= 1 (KKT:154-161)
    m = valid & (ret1d <= 1.0)
    cnt = m.sum(axis=1)
    s = np.where(m, ret1d, 0.0).sum(axis=1)
    mean = np.divide(s, cnt, out=np.zeros_like(s), where=cnt > 0)
    excess = ret1d - mean[:, None]

    tradable = rng.random((T, A)) < tradable_p
    group_id = rng.integers(1, 12, size=A).astype(np.int64)

    def pad(x, fill):
        out = np.full((T, lda), fill, dtype=x.dtype)
        out[:, :A] = x
        return out

    return Panel(dates=dates, ids=ids, close=pad(close, np.nan), volume=pad(volume, np.nan),
                 ret1d=pad(ret1d, np.nan), excess=pad(excess, np.nan),
                 valid=pad(valid, False), tradable=pad(tradable, False), group_id=group_id)


def to_frame(p: Panel):
    """Long DataFrame in the reference's ``merged_df`` schema (``KKT:164-172``), one row per
    present asset-day, date-major order (compute_factors re-sorts it, ``No-talib.py:2``)."""
    import pandas as pd
    tt, aa = np.nonzero(p.valid[:, :p.A])
    df = pd.DataFrame({
        "data_date": p.dates[tt],
        "security_id": p.ids[aa],
        "close_price": p.close[tt, aa],
        "volume": p.volume[tt, aa],
        "ret1d": p.ret1d[tt, aa],
        "excess_ret1d": p.excess[tt, aa],
        "group_id": p.group_id[aa],
        "in_trading_universe": np.where(p.tradable[tt, aa], "Y", "N"),
    })
    return df


def valid_bits(valid: np.ndarray) -> np.ndarray:
    """Pack a ``[T][lda]`` bool mask into ``[ceil(T/64)][lda]`` uint64 words (bit s of word
    ``[c][a]`` = cell ``(64c + s, a)``) -- the mask layout of ``afm_factors_f64``."""
    T, lda = valid.shape
    nc = (T + 63) // 64
    v = np.zeros((nc * 64, lda), dtype=np.uint64)
    v[:T] = valid
    v = v.reshape(nc, 64, lda)
    sh = np.arange(64, dtype=np.uint64)[None, :, None]
    return np.bitwise_or.reduce(v << sh, axis=1).astype(np.uint64)


def unpack_bits(bits: np.ndarray, T: int) -> np.ndarray:
    nc, lda = bits.shape
    sh = np.arange(64, dtype=np.uint64)[None, :, None]
    v = (bits[:, None, :] >> sh) & np.uint64(1)
    return v.reshape(nc * 64, lda)[:T].astype(bool)

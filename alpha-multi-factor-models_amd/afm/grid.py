"""Device-resident calendar-grid panels and the long-DataFrame <-> grid plumbing.

The reference works on a long DataFrame with one row per (security_id, data_date)
(``KKT Yuliang Jiang.py:164-172``).  The engine works on calendar grids in HBM: ``[T][lda]``
fp64 planes (date-major, asset-minor, ``lda`` a multiple of 64) plus a presence bit mask
``[ceil(T/64)][lda]``; windows stay positional per asset because the kernels count only present
days.  torch is used here purely for device memory and indexing (plumbing).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .synthetic import LANES, Panel, round_up


def _torch():
    import torch
    return torch


def pack_bits(valid):
    """``[T][lda]`` bool (torch, device) -> ``[ceil(T/64)][lda]`` int64 words holding the uint64
    presence bits (bit s of word [c][a] = day 64c+s)."""
    torch = _torch()
    T, lda = valid.shape
    nch = (T + 63) // 64
    out = torch.empty((nch, lda), dtype=torch.int64, device=valid.device)
    sh = torch.arange(64, device=valid.device, dtype=torch.int64).view(64, 1)
    step = max(1, (1 << 24) // max(lda * 64, 1))
    for c0 in range(0, nch, step):
        c1 = min(nch, c0 + step)
        v = torch.zeros(((c1 - c0) * 64, lda), dtype=torch.int64, device=valid.device)
        t0, t1 = c0 * 64, min(T, c1 * 64)
        v[: t1 - t0] = valid[t0:t1]
        out[c0:c1] = (v.view(c1 - c0, 64, lda) << sh).sum(dim=1)
    return out


def unpack_bits(bits, T: int):
    torch = _torch()
    nch, lda = bits.shape
    sh = torch.arange(64, device=bits.device, dtype=torch.int64).view(1, 64, 1)
    v = (bits.view(nch, 1, lda) >> sh) & 1
    return v.view(nch * 64, lda)[:T].bool()


@dataclass
class PanelGrid:
    """A panel resident in HBM (the engine's working layout)."""
    dates: np.ndarray          # [T] datetime64[ns] (host)
    ids: np.ndarray            # [A] int64 security ids, ascending (host)
    close: object              # torch [T][lda] float64
    volume: object
    ret1d: object
    excess: object
    valid: object              # torch [T][lda] bool
    vbits: object              # torch [ceil(T/64)][lda] int64 (uint64 bit pattern)
    tradable: object = None    # torch [T][lda] bool
    tbits: object = None       # torch [ceil(T/64)][lda] present AND tradable bits

    @property
    def T(self) -> int:
        return int(self.close.shape[0])

    @property
    def lda(self) -> int:
        return int(self.close.shape[1])

    @property
    def A(self) -> int:
        return len(self.ids)

    @property
    def device(self):
        return self.close.device

    def n_asset_days(self) -> int:
        return int(self.valid.sum().item())

    @classmethod
    def from_panel(cls, p: Panel, device=None) -> "PanelGrid":
        torch = _torch()
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())

        def up(x, dt=torch.float64):
            return torch.from_numpy(np.ascontiguousarray(x)).to(device=dev, dtype=dt)

        valid = up(p.valid, torch.bool)
        trad = up(p.tradable, torch.bool)
        return cls(dates=p.dates, ids=p.ids, close=up(p.close), volume=up(p.volume),
                   ret1d=up(p.ret1d), excess=up(p.excess), valid=valid, vbits=pack_bits(valid),
                   tradable=trad, tbits=pack_bits(trad & valid))

    @classmethod
    def from_frame(cls, df, device=None):
        """Long DataFrame (reference schema) -> (grid, t_idx, a_idx) where row r of ``df`` sits at
        cell (t_idx[r], a_idx[r])."""
        torch = _torch()
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        dates_col = df["data_date"].to_numpy()
        ids_col = df["security_id"].to_numpy()
        dates, t_idx = np.unique(dates_col, return_inverse=True)
        ids, a_idx = np.unique(ids_col, return_inverse=True)
        T, A = len(dates), len(ids)
        lda = round_up(max(A, 1), LANES)
        key = t_idx.astype(np.int64) * lda + a_idx
        if len(np.unique(key)) != len(key):
            raise ValueError("duplicate (data_date, security_id) rows: the calendar grid needs "
                             "one row per security per date (aggregate them first, as "
                             "merge_datasets does at KKT:140)")
        ti = torch.from_numpy(t_idx.astype(np.int64)).to(dev)
        ai = torch.from_numpy(a_idx.astype(np.int64)).to(dev)

        def plane(col):
            g = torch.full((T, lda), float("nan"), dtype=torch.float64, device=dev)
            g[ti, ai] = torch.from_numpy(df[col].to_numpy(np.float64)).to(dev)
            return g

        valid = torch.zeros((T, lda), dtype=torch.bool, device=dev)
        valid[ti, ai] = True
        trad = None
        if "in_trading_universe" in df.columns:
            trad = torch.zeros((T, lda), dtype=torch.bool, device=dev)
            trad[ti, ai] = torch.from_numpy(df["in_trading_universe"].to_numpy() == "Y").to(dev)
        g = cls(dates=np.asarray(dates, dtype="datetime64[ns]"), ids=ids.astype(np.int64),
                close=plane("close_price"), volume=plane("volume"), ret1d=plane("ret1d"),
                excess=plane("excess_ret1d"), valid=valid, vbits=pack_bits(valid), tradable=trad,
                tbits=pack_bits(trad & valid) if trad is not None else None)
        return g, ti, ai

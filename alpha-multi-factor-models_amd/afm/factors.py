"""Factor panel -- drop-in for ``compute_factors`` (No-talib.py:1-93), SURVEY.md §8(a) I0-I16.

``compute_factors(data)`` keeps the reference's pandas-in/pandas-out contract: rows sorted by
(security_id, data_date), the input columns followed by the 98 factor columns in creation
order, the pre-dropna RangeIndex, and ``dropna()`` over every column.  The arithmetic runs in
``afm_factors_f64`` (csrc/factors.hip) on the GPU and is bit-identical to pandas 2.3.3.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .grid import PanelGrid

N_FACTORS = 98
FACTOR_NAMES = (
    [f"SMA_{i}" for i in range(6, 51, 4)]
    + [f"EMA_{i}" for i in range(6, 51, 4)]
    + [f"VWMA_{i}" for i in range(6, 51, 4)]
    + [n for i in range(14, 61, 6) for n in (f"BBANDS_upper_{i}", f"BBANDS_lower_{i}")]
    + [f"MOM_{i}" for i in range(14, 61, 6)]
    + [f"ACCEL_{i}" for i in range(14, 61, 6)]
    + [f"ROCR_{i}" for i in range(14, 61, 6)]
    + [f"MACD_12_{i}" for i in (18, 24, 30)]
    + [f"RSI_{i}" for i in (8, 14, 20)]
    + ["PVT", "OBV", "PSY"]
    + [f"sd_{i}" for i in (3, 5, 15)] + ["sd5_15"]
    + [f"volsd_{i}" for i in (3, 5, 15)] + ["volsd5_15"]
    + ["vol_change", "corr_5", "corr_15", "target", "tmr_ret1d"]
)
COL = {n: i for i, n in enumerate(FACTOR_NAMES)}
TARGET, TMR = COL["target"], COL["tmr_ret1d"]


def factor_panel(grid: PanelGrid, out=None, nanfree=None, finite=None):
    """Run the factor kernel on a device-resident grid.

    Returns ``(out, nanfree)``: ``out`` torch float64 ``[98][T][lda]`` (absent cells NaN or untouched,
    NaN-initialised when allocated here), ``nanfree`` int64 ``[ceil(T/64)][lda]`` presence-and-
    no-NaN-in-96-factors bits (afm.h).  ``finite`` (optional, preallocated like ``nanfree``)
    receives the presence-and-all-96-finite bits."""
    import torch
    ctx = _lib.Context.get(grid.device.index)
    T, lda = grid.T, grid.lda
    if out is None:
        out = torch.full((N_FACTORS, T, lda), float("nan"), dtype=torch.float64,
                         device=grid.device)
    if nanfree is None:
        nanfree = torch.zeros(((T + 63) // 64, lda), dtype=torch.int64, device=grid.device)
    assert out.shape == (N_FACTORS, T, lda) and out.dtype == torch.float64
    assert nanfree.shape == ((T + 63) // 64, lda)
    P = _lib.ptr
    _lib.check(_lib.lib().afm_factors_f64(
        ctx.bind_stream(), T, grid.A, lda, P(grid.close), P(grid.volume), P(grid.ret1d),
        P(grid.excess), P(grid.vbits), P(out), P(nanfree),
        P(finite) if finite is not None else None), "afm_factors_f64")
    return out, nanfree


def compute_factors(data):
    """Drop-in for ``compute_factors(data)`` (No-talib.py:1-93)."""
    import pandas as pd
    data = data.sort_values(by=["security_id", "data_date"])           # NT:2
    grid, ti, ai = PanelGrid.from_frame(data)
    out, _ = factor_panel(grid)
    vals = out[:, ti, ai].T.contiguous().cpu().numpy()                # rows in (id, date) order
    base = data.reset_index(drop=True)                                # concat(ignore_index) NT:32
    res = pd.concat([base, pd.DataFrame(vals, columns=FACTOR_NAMES)], axis=1)
    return res.dropna()                                               # NT:33

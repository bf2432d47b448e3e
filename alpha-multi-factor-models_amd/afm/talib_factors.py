"""The talib factor variant -- drop-in for the reference's second ``compute_factors``
(KKT Yuliang Jiang.py:176-270), SURVEY.md §8(f) rank 3.

106 columns per row, in the reference's creation order: TA-Lib SMA / EMA / VSMA (SMA of
volume * close), BBANDS upper / middle / lower, MOM, ACCEL, ROCR, MACD_12_i, RSI_i, PVT (volume *
pct_change, no cumsum), TA-Lib OBV, PSY, sd, volsd, vol_change, corr, target, tmr_ret1d.
The TA-Lib columns run in ``afm_talib_factors_f64`` (csrc/talib.hip); MOM (TA-Lib MOM is the
same subtraction as pandas' diff) and the pandas columns come from ``afm_factors_f64``, so they
are the pandas-exact values of the No-talib path.  TA-Lib is not installed here: its semantics are
restated from its C core (see csrc/talib.hip) and parity with TA-Lib itself is unpinned."""
from __future__ import annotations

import numpy as np

from . import _lib
from .factors import COL, factor_panel
from .grid import PanelGrid

TALIB_COLS = 68
_TL = ([f"SMA_{i}" for i in range(6, 51, 4)] + [f"EMA_{i}" for i in range(6, 51, 4)]
       + [f"VSMA_{i}" for i in range(6, 51, 4)]
       + [f"BBANDS_{b}_{i}" for i in range(14, 61, 6) for b in ("upper", "middle", "lower")]
       + [f"MACD_12_{i}" for i in (18, 24, 30)] + [f"RSI_{i}" for i in (8, 14, 20)]
       + ["PVT", "OBV"])
TALIB_PLANE = {n: i for i, n in enumerate(_TL)}
TALIB_NAMES = (
    [f"SMA_{i}" for i in range(6, 51, 4)] + [f"EMA_{i}" for i in range(6, 51, 4)]
    + [f"VSMA_{i}" for i in range(6, 51, 4)]
    + [f"BBANDS_{b}_{i}" for i in range(14, 61, 6) for b in ("upper", "middle", "lower")]
    + [f"MOM_{i}" for i in range(14, 61, 6)] + [f"ACCEL_{i}" for i in range(14, 61, 6)]
    + [f"ROCR_{i}" for i in range(14, 61, 6)]
    + [f"MACD_12_{i}" for i in (18, 24, 30)] + [f"RSI_{i}" for i in (8, 14, 20)]
    + ["PVT", "OBV", "PSY"] + [f"sd_{i}" for i in (3, 5, 15)] + ["sd5_15"]
    + [f"volsd_{i}" for i in (3, 5, 15)] + ["volsd5_15"]
    + ["vol_change", "corr_5", "corr_15", "target", "tmr_ret1d"])
assert len(TALIB_NAMES) == 106 and len(_TL) == TALIB_COLS


def talib_panel(grid: PanelGrid, out=None):
    """The 68 TA-Lib planes ``[68][T][lda]`` (NaN where absent when allocated here)."""
    import torch
    T, lda = grid.T, grid.lda
    if out is None:
        out = torch.full((TALIB_COLS, T, lda), float("nan"), dtype=torch.float64,
                         device=grid.device)
    assert out.shape == (TALIB_COLS, T, lda) and out.dtype == torch.float64
    ctx = _lib.Context.get(grid.device.index)
    P = _lib.ptr
    _lib.check(_lib.lib().afm_talib_factors_f64(ctx.bind_stream(), T, grid.A, lda, P(grid.close),
                                                P(grid.volume), P(grid.vbits), P(out)),
               "afm_talib_factors_f64")
    return out


def compute_factors_talib(data):
    """Drop-in for the talib ``compute_factors(data)`` (KKT:176-270)."""
    import pandas as pd
    import torch
    data = data.sort_values(by=["security_id", "data_date"])           # KKT:178
    grid, ti, ai = PanelGrid.from_frame(data)
    fac, _ = factor_panel(grid)
    tl = talib_panel(grid)
    src = []
    for n in TALIB_NAMES:
        src.append(tl[TALIB_PLANE[n]] if n in TALIB_PLANE else fac[COL[n]])
    vals = torch.stack([s[ti, ai] for s in src], dim=1).cpu().numpy()
    base = data.reset_index(drop=True)                                # concat(ignore_index) KKT:266
    res = pd.concat([base, pd.DataFrame(vals, columns=TALIB_NAMES)], axis=1)
    return res.dropna()                                               # KKT:268

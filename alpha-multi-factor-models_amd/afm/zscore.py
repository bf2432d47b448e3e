"""Per-security z-score and train/valid/test split -- the notebook cells between the factor build
and the models (``KKT Yuliang Jiang.py:424-458``).

* ``zscore_grid`` -- the engine form: train-window ``groupby('security_id').mean()/.std()``
  over device-resident factor planes (``afm_zscore_stats_f64``), then ``(x - mu) / sigma``,
  ``inf -> NaN`` and the ``dropna()`` row bits (``afm_zscore_apply_f64``), in place or into new
  planes.  Kernels in csrc/zscore.hip.
* ``split_zscore`` -- the drop-in for the cells themselves: ``all_df`` (indexed by
  (data_date, security_id), KKT:275) in, the six frames ``df_{train,valid,test}_{x,y}`` out,
  with the reference's column set (``Index.difference``, KKT:433-443), row order
  (``sort_index``) and values.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .grid import pack_bits
from .synthetic import LANES, round_up

# KKT:433-443: every column except these is a feature (tmr_ret1d included, as in the reference)
EXCLUDED = ("close_price", "excess_ret1d", "group_id", "in_trading_universe", "ret1d", "volume",
            "target")


def zscore_grid(planes, lda: int, cols, bits, train, apply=None, out=None, out_cols=None,
                col_stride: int | None = None):
    """Z-score the feature planes ``planes[cols[k]]`` (``[T][lda]`` fp64 each).

    ``bits`` are the row bits (``[ceil(T/64)][lda]``), ``train = (t0, t1)`` the date range of the
    statistics (KKT:446-447), ``apply = (a0, a1)`` the range transformed (default: every date).
    ``out=None`` transforms in place; otherwise output column k goes to ``out[out_cols[k]]``
    (default ``out_cols = range(K)``).  Returns ``(mu, sd, keep)``: ``[K][lda]`` statistics and
    the kept-row bits of the applied range (KKT:449-451)."""
    import torch
    dev = planes.device
    T = int(planes.shape[-2])
    cs = int(col_stride if col_stride is not None else planes.stride(0))
    cols_t = torch.as_tensor(np.asarray(cols, dtype=np.int32), device=dev)
    K = int(cols_t.numel())
    if out is None:
        out, ocols_t, ocs = planes, cols_t, cs
    else:
        ocols = np.arange(K) if out_cols is None else out_cols
        ocols_t = torch.as_tensor(np.asarray(ocols, dtype=np.int32), device=dev)
        ocs = int(out.stride(0))
    a0, a1 = (0, T) if apply is None else apply
    mu = torch.empty((K, lda), dtype=torch.float64, device=dev)
    sd = torch.empty((K, lda), dtype=torch.float64, device=dev)
    keep = torch.zeros_like(bits)
    ctx = _lib.Context.get(dev.index)
    P, L = _lib.ptr, _lib.lib()
    _lib.check(L.afm_zscore_stats_f64(ctx.bind_stream(), P(planes), cs, T, lda, P(cols_t), K,
                                      P(bits), int(train[0]), int(train[1]), P(mu), P(sd)),
               "afm_zscore_stats_f64")
    _lib.check(L.afm_zscore_apply_f64(ctx.bind_stream(), P(planes), cs, T, lda, P(cols_t), K,
                                      P(bits), int(a0), int(a1), P(mu), P(sd), P(out), ocs,
                                      P(ocols_t), P(keep)), "afm_zscore_apply_f64")
    return mu, sd, keep


def split_zscore(all_df, train_edate="20151231", valid_edate="20161231"):
    """Drop-in for KKT:424-458 -> dict with ``df_train_x, df_valid_x, df_test_x, df_train_y,
    df_valid_y, df_test_y``.

    ``all_df``: the factor frame indexed by (data_date, security_id), sorted (KKT:275).  The
    ``.loc`` date slices are inclusive at both ends, so the boundary dates belong to two splits,
    exactly as in the reference."""
    import pandas as pd
    import torch
    dev = torch.device("cuda", torch.cuda.current_device())
    te, ve = pd.to_datetime(train_edate), pd.to_datetime(valid_edate)
    xcols = list(all_df.columns.difference(list(EXCLUDED)))
    dates_col = all_df.index.get_level_values(0).values
    ids_col = all_df.index.get_level_values(1).values
    dates, t_idx = np.unique(dates_col, return_inverse=True)
    ids, a_idx = np.unique(ids_col, return_inverse=True)
    T, K = len(dates), len(xcols)
    lda = round_up(max(len(ids), 1), LANES)
    ti = torch.from_numpy(t_idx.astype(np.int64)).to(dev)
    ai = torch.from_numpy(a_idx.astype(np.int64)).to(dev)
    planes = torch.full((K, T, lda), float("nan"), dtype=torch.float64, device=dev)
    planes[:, ti, ai] = torch.from_numpy(all_df[xcols].to_numpy(np.float64).T.copy()).to(dev)
    valid = torch.zeros((T, lda), dtype=torch.bool, device=dev)
    valid[ti, ai] = True
    bits = pack_bits(valid)
    d64 = dates.astype("datetime64[ns]")
    t_tr = int(np.searchsorted(d64, np.datetime64(te, "ns"), side="right"))   # date <= te
    mu, sd, keep = zscore_grid(planes, lda, range(K), bits, train=(0, t_tr))
    from .grid import unpack_bits
    kept = unpack_bits(keep, T)
    target = None
    if "target" in all_df.columns:
        target = torch.full((T, lda), float("nan"), dtype=torch.float64, device=dev)
        target[ti, ai] = torch.from_numpy(all_df["target"].to_numpy(np.float64)).to(dev)
    ranges = {"train": (None, te), "valid": (te, ve), "test": (ve, None)}
    res = {}
    for nm, (lo, hi) in ranges.items():
        tlo = 0 if lo is None else int(np.searchsorted(d64, np.datetime64(lo, "ns"), side="left"))
        thi = T if hi is None else int(np.searchsorted(d64, np.datetime64(hi, "ns"), side="right"))
        tt, aa = torch.nonzero(kept[tlo:thi], as_tuple=True)       # (date, id) order
        tt = tt + tlo
        idx = pd.MultiIndex.from_arrays([dates[tt.cpu().numpy()], ids[aa.cpu().numpy()]],
                                        names=all_df.index.names)
        vals = planes[:, tt, aa].T.contiguous().cpu().numpy()
        res[f"df_{nm}_x"] = pd.DataFrame(vals, index=idx, columns=xcols)
        if target is not None:
            res[f"df_{nm}_y"] = pd.DataFrame({"target": target[tt, aa].cpu().numpy()}, index=idx)
    return res

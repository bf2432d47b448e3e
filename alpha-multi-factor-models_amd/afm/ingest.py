"""Ingest / clean -- drop-in for ``merge_datasets`` (KKT Yuliang Jiang.py:113-166), SURVEY.md
§8(f) rank 2.

The reference builds the long panel the factor path consumes (``merged_df``, KKT:164-172):

1. each ``data_set_N`` file: ``groupby(['data_date', 'security_id']).mean().drop_duplicates()``
   (KKT:133-140; note ``drop_duplicates`` compares values only, so a row whose values equal an
   earlier row's is dropped -- kept as is);
2. outer concat on (date, id) (KKT:143);
3. per security, forward fill in date order (KKT:145);
4. per date, NaN cells take the column mean over that date's rows (KKT:147);
5. the security reference rows with ``ret1d <= 1``, ``excess_ret1d = ret1d - mean`` per date
   (KKT:149-161), left-merged on (date, id), then ``dropna`` (KKT:163-166).

Steps 3-5's arithmetic -- the per-security scans and the per-date means, which the reference runs
as Python lambdas per group -- run on the GPU (``afm_ffill_f64``, ``afm_date_mean_fill_f64``,
``afm_group_demean_f64``) on the calendar-grid layout; CSV parsing, the per-file dedupe and the
final key merge stay in pandas (I/O and joins, with the reference's exact row / index / dtype
semantics).  Bit-exact with the reference (tests/golden/ingest_*.npz)."""
from __future__ import annotations

import re

import numpy as np

from . import _lib
from .grid import pack_bits
from .synthetic import round_up

SEC_REF_FILES = ("security_reference_data_w_ret1d_1.csv", "security_reference_data_w_ret1d_2.csv")


def _dataset_number(name: str) -> int:
    return int(re.search(r"data_set_(\d+)", name).group(1))


def load_dataset(file: str):
    """One ``data_set_N`` file as the reference reads it (KKT:133-140)."""
    import pandas as pd
    compression = "zip" if file.endswith(".zip") else None
    df = pd.read_csv(file, compression=compression)
    df["data_date"] = pd.to_datetime(df["data_date"].apply(str))
    return df.groupby(["data_date", "security_id"]).mean().drop_duplicates()


def _dev(device):
    import torch
    return device if device is not None else torch.device("cuda", torch.cuda.current_device())


def fill_panel(values: np.ndarray, t_idx: np.ndarray, a_idx: np.ndarray, T: int, A: int,
               device=None) -> np.ndarray:
    """Steps 3-4 on the GPU: ``values`` [rows][K] at grid cells (t_idx, a_idx) -> the filled
    values in the same row order."""
    import torch
    dev = _dev(device)
    K = values.shape[1]
    lda = round_up(max(A, 1))
    ti = torch.from_numpy(t_idx.astype(np.int64)).to(dev)
    ai = torch.from_numpy(a_idx.astype(np.int64)).to(dev)
    planes = torch.full((K, T, lda), float("nan"), dtype=torch.float64, device=dev)
    planes[:, ti, ai] = torch.from_numpy(np.ascontiguousarray(values.T)).to(dev)
    valid = torch.zeros((T, lda), dtype=torch.bool, device=dev)
    valid[ti, ai] = True
    bits = pack_bits(valid)
    scratch = torch.empty_like(planes)
    ctx = _lib.Context.get(dev.index)
    h = ctx.bind_stream()
    L, P = _lib.lib(), _lib.ptr
    _lib.check(L.afm_ffill_f64(h, K, T, lda, P(planes), P(bits)), "afm_ffill_f64")
    _lib.check(L.afm_date_mean_fill_f64(h, K, T, A, lda, P(planes), P(bits), P(scratch)),
               "afm_date_mean_fill_f64")
    return planes[:, ti, ai].T.contiguous().cpu().numpy()


def group_demean(x: np.ndarray, offsets: np.ndarray, device=None) -> np.ndarray:
    """x - mean(x) per group of consecutive rows (``afm_group_demean_f64``)."""
    import torch
    dev = _dev(device)
    n = len(x)
    if n == 0:
        return x.astype(np.float64)
    xt = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).to(dev)
    off = torch.from_numpy(np.ascontiguousarray(offsets, dtype=np.int64)).to(dev)
    out = torch.empty_like(xt)
    scratch = torch.empty_like(xt)
    ctx = _lib.Context.get(dev.index)
    _lib.check(_lib.lib().afm_group_demean_f64(ctx.bind_stream(), len(offsets) - 1, _lib.ptr(off),
                                               int(np.diff(offsets).max()), _lib.ptr(xt),
                                               _lib.ptr(out), _lib.ptr(scratch)),
               "afm_group_demean_f64")
    return out.cpu().numpy()


def security_reference(files=SEC_REF_FILES, device=None):
    """The reference data with ``excess_ret1d`` (KKT:149-161): rows with ``ret1d <= 1``, grouped
    by date (ascending; file order within a date), columns ``data_date``, ``security_id``, then
    the other columns sorted by name (``columns.difference``)."""
    import pandas as pd
    sec_ref = pd.concat([pd.read_csv(f) for f in files])
    sec_ref = sec_ref[sec_ref["ret1d"] <= 1]
    order = np.argsort(sec_ref["data_date"].to_numpy(), kind="stable")
    s = sec_ref.iloc[order].reset_index(drop=True)
    d = s["data_date"].to_numpy()
    starts = np.flatnonzero(np.r_[True, d[1:] != d[:-1]]) if len(d) else np.zeros(0, np.int64)
    offsets = np.r_[starts, len(d)].astype(np.int64)
    s["excess_ret1d"] = group_demean(s["ret1d"].to_numpy(np.float64), offsets, device)
    rest = s.columns.difference(["data_date", "security_id"])
    out = pd.concat([s[["data_date", "security_id"]], s[rest]], axis=1)
    out["data_date"] = pd.to_datetime(out["data_date"].apply(str))
    return out


def merge_datasets(files: list, sec_ref_files=SEC_REF_FILES, device=None):
    """Drop-in for ``merge_datasets(files)`` (KKT:113-166)."""
    import pandas as pd
    frames = [load_dataset(f) for f in sorted(files, key=_dataset_number)]
    merged = pd.concat(frames, axis=1, join="outer")
    cols = list(merged.columns)
    dcol = merged.index.get_level_values(0).to_numpy()
    icol = merged.index.get_level_values(1).to_numpy()
    dates, t_idx = np.unique(dcol, return_inverse=True)
    ids, a_idx = np.unique(icol, return_inverse=True)
    order = np.lexsort((a_idx, t_idx))                # rows of steps 3-4: (date, security) order
    t_idx, a_idx = t_idx[order], a_idx[order]
    vals = merged.to_numpy(np.float64)[order]
    filled = fill_panel(vals, t_idx, a_idx, len(dates), len(ids), device)
    m = pd.DataFrame({"data_date": dates[t_idx], "security_id": ids[a_idx]})
    for j, c in enumerate(cols):
        m[c] = filled[:, j]
    sec_ref = security_reference(sec_ref_files, device)
    out = pd.merge(m, sec_ref, on=["data_date", "security_id"], how="left")
    return out.dropna()

"""ORACLE -- test infrastructure only.  CPU restatement of ``merge_datasets``
(KKT Yuliang Jiang.py:113-166), pinned by the reference's own outputs
(tests/golden/make_ingest_golden.py -> tests/golden/ingest_*.npz).

The reference's per-group lambdas are restated as explicit loops:
* KKT:145 ``groupby('security_id').apply(sort_values('data_date').ffill())`` -> per security,
  in date order, a NaN takes the last non-NaN value;
* KKT:147 ``groupby('data_date').apply(fillna(group.mean()))`` -> per date and column, pandas
  nanmean over the date's rows in security order = ``np.add.reduce`` (numpy pairwise) of the
  contiguous values with NaN -> 0, divided by the non-NaN count (verified against the reference:
  a sequential sum mismatches);
* KKT:157-158 ``x['ret1d'] - x['ret1d'].mean()`` per date over the reference rows in file order.
"""
from __future__ import annotations

import re

import numpy as np
import pandas as pd


def _load(file):                                               # KKT:133-140
    df = pd.read_csv(file, compression="zip" if file.endswith(".zip") else None)
    df["data_date"] = pd.to_datetime(df["data_date"].apply(str))
    return df.groupby(["data_date", "security_id"]).mean().drop_duplicates()


def _nanmean(v: np.ndarray) -> float:
    cnt = int((~np.isnan(v)).sum())
    if cnt == 0:
        return np.nan
    return np.add.reduce(np.ascontiguousarray(np.where(np.isnan(v), 0.0, v))) / float(cnt)


def merge_datasets(files, sec_ref_files=("security_reference_data_w_ret1d_1.csv",
                                         "security_reference_data_w_ret1d_2.csv")):
    files = sorted(files, key=lambda x: int(re.search(r"data_set_(\d+)", x).group(1)))
    merged = pd.concat([_load(f) for f in files], axis=1, join="outer").reset_index()
    cols = [c for c in merged.columns if c not in ("data_date", "security_id")]
    merged = merged.sort_values(["data_date", "security_id"], kind="stable").reset_index(drop=True)
    d = merged["data_date"].to_numpy()
    s = merged["security_id"].to_numpy()
    V = merged[cols].to_numpy(np.float64).copy()
    # KKT:145 ffill per security in date order
    for sid in np.unique(s):
        rows = np.flatnonzero(s == sid)                        # date order (frame is sorted)
        for j in range(V.shape[1]):
            last = np.nan
            for r in rows:
                if np.isnan(V[r, j]):
                    V[r, j] = last
                else:
                    last = V[r, j]
    # KKT:147 per-date mean fill
    starts = np.flatnonzero(np.r_[True, d[1:] != d[:-1]])
    for lo, hi in zip(starts, np.r_[starts[1:], len(d)]):
        for j in range(V.shape[1]):
            v = V[lo:hi, j]
            if np.isnan(v).any():
                V[lo:hi, j] = np.where(np.isnan(v), _nanmean(v), v)
    m = pd.DataFrame({"data_date": d, "security_id": s})
    for j, c in enumerate(cols):
        m[c] = V[:, j]
    # KKT:149-161 security reference + excess return
    ref = pd.concat([pd.read_csv(f) for f in sec_ref_files])
    ref = ref[ref["ret1d"] <= 1]
    ref = ref.iloc[np.argsort(ref["data_date"].to_numpy(), kind="stable")].reset_index(drop=True)
    dd = ref["data_date"].to_numpy()
    ex = np.empty(len(ref))
    r1 = ref["ret1d"].to_numpy(np.float64)
    st = np.flatnonzero(np.r_[True, dd[1:] != dd[:-1]]) if len(dd) else np.zeros(0, np.int64)
    for lo, hi in zip(st, np.r_[st[1:], len(dd)]):
        ex[lo:hi] = r1[lo:hi] - _nanmean(r1[lo:hi])
    ref["excess_ret1d"] = ex
    rest = ref.columns.difference(["data_date", "security_id"])
    ref = pd.concat([ref[["data_date", "security_id"]], ref[rest]], axis=1)
    ref["data_date"] = pd.to_datetime(ref["data_date"].apply(str))
    return pd.merge(m, ref, on=["data_date", "security_id"], how="left").dropna()

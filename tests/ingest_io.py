"""Synthetic CSV sets for the ingest row and their (de)serialisation as plain arrays (shared by
tests/golden/make_ingest_golden.py and tests/test_ingest.py)."""
import os

import numpy as np
import pandas as pd


def synth_csvs(seed: int, n_ids: int, n_dates: int) -> dict:
    """{file name: DataFrame} in the reference's schemas (KKT:45-56, 133-151)."""
    rng = np.random.default_rng(seed)
    dates = pd.bdate_range("2019-01-01", periods=n_dates)
    di = np.array([int(x.strftime("%Y%m%d")) for x in dates], dtype=np.int64)
    ids = np.sort(rng.choice(np.arange(10, 10 * n_ids * 3), n_ids, replace=False))
    first = rng.integers(0, n_dates // 3, n_ids)
    out = {}
    for k, (p, dec) in enumerate([(0.7, None), (0.5, 2), (0.8, None)], start=1):
        tt, aa = np.nonzero((rng.random((n_dates, n_ids)) < p)
                            & (np.arange(n_dates)[:, None] >= first[None, :]))
        v = rng.normal(size=len(tt)) * 10.0 ** rng.uniform(-3, 3, len(tt))
        if dec is not None:
            v = np.round(v, dec)                      # value ties -> drop_duplicates drops rows
        df = pd.DataFrame({"data_date": di[tt], "security_id": ids[aa], f"value_{k}": v})
        if k == 2:
            df.loc[df["data_date"] == di[n_dates // 2], f"value_{k}"] = np.nan   # a column gap
            df = pd.concat([df, df.iloc[:5].assign(**{f"value_{k}": 7.25})])     # dup keys
        name = f"data_set_{k}.csv" + (".zip" if k == 3 else "")
        out[name] = df.reset_index(drop=True)
    tt, aa = np.nonzero(rng.random((n_dates, n_ids)) < 0.93)
    ref = pd.DataFrame({"data_date": di[tt], "security_id": ids[aa],
                        "close_price": rng.uniform(5, 50, len(tt)),
                        "volume": rng.integers(1_000, 90_000, len(tt)).astype(np.float64),
                        "ret1d": rng.normal(0, 0.02, len(tt)),
                        "group_id": rng.integers(1, 12, len(tt)),
                        "in_trading_universe": np.where(rng.random(len(tt)) < 0.85, "Y", "N")})
    ref.loc[rng.random(len(ref)) < 0.01, "ret1d"] = 1.7
    # unsorted within a date: shuffle, then stable-sort by date only
    ref = ref.iloc[rng.permutation(len(ref))]
    ref = ref.iloc[np.argsort(ref["data_date"].to_numpy(), kind="stable")].reset_index(drop=True)
    half = len(ref) // 2
    out["security_reference_data_w_ret1d_1.csv"] = ref.iloc[:half].reset_index(drop=True)
    out["security_reference_data_w_ret1d_2.csv"] = ref.iloc[half:].reset_index(drop=True)
    return out


def write_csvs(files: dict, d: str):
    for name, df in files.items():
        path = os.path.join(d, name)
        if name.endswith(".zip"):
            df.to_csv(path, index=False,
                      compression={"method": "zip", "archive_name": name[:-4]})
        else:
            df.to_csv(path, index=False)


def read_fixture(npz) -> dict:
    files = {}
    for key in npz.files:
        tag, rest = key.split("|", 1)
        if tag != "in":
            continue
        fname, col = rest.split("|")
        files.setdefault(fname, {})[col] = npz[key]
    return {f: pd.DataFrame(cols) for f, cols in files.items()}


def frame_arrays(df) -> dict:
    out = {"index": df.index.to_numpy(np.int64), "columns": np.array(list(df.columns)),
           "dtypes": np.array([str(t) for t in df.dtypes])}
    for c in df.columns:
        v = df[c]
        out[f"col:{c}"] = v.to_numpy("int64") if str(v.dtype).startswith("datetime") else plain(v)
    return out


def plain(v) -> np.ndarray:
    """Column -> array without object dtype (npz stays pickle-free)."""
    a = np.asarray(v)
    return a.astype(str) if a.dtype == object else a


def fixture_frame(npz) -> dict:
    return {k[4:]: npz[k] for k in npz.files if k.startswith("out|")}

"""Ingest / clean row: ``merge_datasets`` (KKT:113-166) -- the oracle
(CPU) and afm.merge_datasets (GPU fill / demean kernels) against the reference's own outputs on
the same CSV sets (tests/golden/ingest_*.npz, made by tests/golden/make_ingest_golden.py).
Bar: identical frames -- index labels, column order, dtypes, every value bit for bit."""
import os

import numpy as np
import pytest

from ingest_io import fixture_frame, frame_arrays, read_fixture, write_csvs

CASES = ["basic", "wide"]


def _run(fn, golden_dir, case, tmp_path, monkeypatch):
    z = np.load(os.path.join(golden_dir, f"ingest_{case}.npz"))
    files = read_fixture(z)
    write_csvs(files, str(tmp_path))
    monkeypatch.chdir(tmp_path)
    out = fn([f for f in os.listdir() if "data_set" in f])
    return frame_arrays(out), fixture_frame(z)


def _assert_same(got, want):
    assert list(got["columns"]) == list(want["columns"])
    assert list(got["dtypes"]) == list(want["dtypes"])
    assert np.array_equal(got["index"], want["index"])
    for c in want["columns"]:
        a, b = got[f"col:{c}"], want[f"col:{c}"]
        if a.dtype.kind == "f":
            assert np.array_equal(a, b, equal_nan=True), c
        else:
            assert np.array_equal(a.astype(b.dtype), b), c


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference(golden_dir, case, tmp_path, monkeypatch):
    import warnings

    import oracle.ingest
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        got, want = _run(oracle.ingest.merge_datasets, golden_dir, case, tmp_path, monkeypatch)
    _assert_same(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_merge_datasets_matches_reference(golden_dir, case, tmp_path, monkeypatch):
    import afm.ingest
    got, want = _run(afm.ingest.merge_datasets, golden_dir, case, tmp_path, monkeypatch)
    _assert_same(got, want)


@pytest.mark.gpu
def test_fill_kernels_vs_oracle_large():
    """Per-date means over > 65k-leaf-free but multi-leaf dates (A = 5000) and long ffill runs."""
    import oracle.ingest as oi
    from afm.ingest import fill_panel
    rng = np.random.default_rng(3)
    T, A, K = 40, 5000, 3
    tt, aa = np.nonzero(rng.random((T, A)) < 0.7)
    vals = rng.normal(size=(len(tt), K)) * 10.0 ** rng.uniform(-4, 4, (len(tt), K))
    vals[rng.random(vals.shape) < 0.3] = np.nan
    got = fill_panel(vals, tt, aa, T, A)
    want = vals.copy()
    for a in range(A):                                      # ffill per security
        r = np.flatnonzero(aa == a)
        for j in range(K):
            last = np.nan
            for i in r:
                if np.isnan(want[i, j]):
                    want[i, j] = last
                else:
                    last = want[i, j]
    for t in range(T):                                      # date means
        r = np.flatnonzero(tt == t)
        for j in range(K):
            v = want[r, j]
            if np.isnan(v).any():
                want[r, j] = np.where(np.isnan(v), oi._nanmean(v), v)
    assert np.array_equal(got, want, equal_nan=True)

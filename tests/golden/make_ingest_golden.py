"""Golden vectors for the ingest / clean row: runs the REFERENCE's
``merge_datasets`` (KKT Yuliang Jiang.py:113-166, extracted with ``ast`` and exec'd with pd, np,
re, os -- its source is read at run time, never copied) on synthetic CSV sets written to a temp
directory, and stores the CSV contents and the returned frame as arrays.  The synthetic files
exercise: duplicated (date, id) rows, value ties that ``drop_duplicates`` removes, a zip file,
holes before a security's first value (date-mean fill), a value column with no value on a date,
``ret1d > 1`` rows, reference rows unsorted within a date, and keys missing from the reference.
Run from the repo root: python tests/golden/make_ingest_golden.py"""
import ast
import os
import re
import sys
import tempfile
import warnings

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from ingest_io import frame_arrays, plain, synth_csvs, write_csvs  # noqa: E402

KKT = "/root/reference/KKT Yuliang Jiang.py"


def load_merge_datasets():
    src = open(KKT).read()
    ns = {"pd": pd, "np": np, "re": re, "os": os}
    for n in ast.parse(src).body:
        if isinstance(n, ast.FunctionDef) and n.name == "merge_datasets":
            exec(compile(ast.get_source_segment(src, n), f"KKT:{n.lineno}", "exec"), ns)
    return ns["merge_datasets"]


def main():
    merge = load_merge_datasets()
    for name, kw in {"basic": dict(seed=1, n_ids=120, n_dates=60),
                     "wide": dict(seed=2, n_ids=700, n_dates=20)}.items():
        files = synth_csvs(**kw)
        cwd = os.getcwd()
        with tempfile.TemporaryDirectory() as d:
            write_csvs(files, d)
            os.chdir(d)
            try:
                with warnings.catch_warnings():
                    warnings.simplefilter("ignore")
                    out = merge([f for f in os.listdir() if "data_set" in f])
            finally:
                os.chdir(cwd)
        arrs = {}
        for fname, df in files.items():
            for c in df.columns:
                arrs[f"in|{fname}|{c}"] = plain(df[c])
        arrs.update({f"out|{k}": v for k, v in frame_arrays(out).items()})
        np.savez_compressed(os.path.join(HERE, f"ingest_{name}.npz"), **arrs)


if __name__ == "__main__":
    main()

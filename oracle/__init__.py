"""ORACLE -- test infrastructure only.

CPU restatement of the reference hot path,
used ONLY by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg, and
there only as the checker (or the timed CPU baseline).  The product package
(``alpha-multi-factor-models_amd/afm``) never imports this module and has no CPU fallback.

Parity pin: every function here is checked against golden vectors produced by running the
reference itself (``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``;
``tests/test_oracle_golden.py``).  Exceptions, where the reference has no deterministic target,
are stated per function (the exact box-QP weight solve replaces SLSQP).

Layout: ``factors_oracle.c`` / ``xs_oracle.c`` / ``lasso_oracle.c`` / ``talib_oracle.c`` (plain C, gcc, no FMA contraction) built into
``oracle/build/liboracle.so`` by ``oracle/Makefile``; the pandas-shaped drivers are below and in
``oracle/xs.py`` / ``oracle/portfolio.py``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

# No-talib.py creation order (No-talib.py:9-91)
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
assert len(FACTOR_NAMES) == 98

_lib = None


def build() -> str:
    """Compile the C restatement (gcc) -- building the checker is not using it."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        i64 = ctypes.c_int64
        L.oracle_factors_panel.argtypes = [i64, P, P, P, P, P, P]
        L.oracle_factors_panel.restype = ctypes.c_int
        L.oracle_factors_series.argtypes = [i64, P, P, P, P, P]
        L.oracle_np_sum.argtypes = [i64, P]
        L.oracle_np_sum.restype = ctypes.c_double
        L.oracle_nancorr_pair.argtypes = [i64, P, P]
        L.oracle_nancorr_pair.restype = ctypes.c_double
        L.oracle_group_corr.argtypes = [i64, P, P, P, P]
        L.oracle_group_mean.argtypes = [i64, P, P, i64, P, P, P, P]
        d = ctypes.c_double
        L.oracle_lasso_gram.argtypes = [ctypes.c_int, P, P, d, d, d, ctypes.c_int, d,
                                        ctypes.c_int, P, P, P]
        L.oracle_talib_panel.argtypes = [i64, P, P, P, P, P]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def factors_long(offsets: np.ndarray, close, volume, ret1d, excess) -> np.ndarray:
    """Rows sorted by (security, date), CSR ``offsets`` -> ``[n_rows][98]`` factor block."""
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    cols = [np.ascontiguousarray(x, dtype=np.float64) for x in (close, volume, ret1d, excess)]
    n = int(offsets[-1])
    out = np.empty((n, 98), dtype=np.float64)
    rc = lib().oracle_factors_panel(len(offsets) - 1, _p(offsets), *[_p(c) for c in cols], _p(out))
    if rc:
        raise MemoryError("oracle_factors_panel")
    return out


def compute_factors(data):
    """No-talib.py:1-93 restated: sort by (security_id, data_date) (NT:2), per-security factors
    (NT:5-91), concat with a fresh RangeIndex (NT:32), dropna over every column (NT:33)."""
    import pandas as pd
    data = data.sort_values(by=["security_id", "data_date"])
    sid = data["security_id"].to_numpy()
    starts = np.flatnonzero(np.r_[True, sid[1:] != sid[:-1]])
    offsets = np.r_[starts, len(sid)].astype(np.int64)
    fac = factors_long(offsets, data["close_price"].to_numpy(np.float64),
                       data["volume"].to_numpy(np.float64), data["ret1d"].to_numpy(np.float64),
                       data["excess_ret1d"].to_numpy(np.float64))
    base = data.reset_index(drop=True)
    out = pd.concat([base, pd.DataFrame(fac, columns=FACTOR_NAMES)], axis=1)
    return out.dropna()


def lasso_gram(Q, q, ynorm2: float, alpha_n: float, *, max_iter: int = 1000, tol: float = 1e-4,
               positive: bool = False):
    """sklearn enet_coordinate_descent_gram restated (oracle/lasso_oracle.c, l2 weight 0):
    -> (w, gap, tol * y'y, n_iter) on centered moments Q = X'X, q = X'y, ynorm2 = y'y."""
    Q = np.ascontiguousarray(Q, dtype=np.float64)
    q = np.ascontiguousarray(q, dtype=np.float64)
    p = len(q)
    w = np.zeros(p)
    H = np.zeros(p)
    info = np.zeros(3)
    lib().oracle_lasso_gram(p, _p(Q), _p(q), float(ynorm2), float(alpha_n), 0.0, int(max_iter),
                            float(tol), int(bool(positive)), _p(w), _p(H), _p(info))
    return w, float(info[0]), float(info[1]), int(info[2])


def centered_moments(G, n_index=True):
    """Shifted moments G' [p+2][p+2] of [1, x, y] (afm's Gram layout) -> (n, Q, q, y'y): the
    centered cross-products C = G'[1:,1:] - outer(G'[0,1:], G'[0,1:]) / n."""
    G = np.asarray(G, dtype=np.float64)
    n = G[0, 0]
    g0 = G[0, 1:]
    C = G[1:, 1:] - np.outer(g0, g0) / n
    p = G.shape[0] - 2
    return n, C[:p, :p], C[:p, p], C[p, p]


TALIB_COLS = 68


def talib_factors_long(offsets: np.ndarray, close, volume) -> np.ndarray:
    """TA-Lib columns of the talib variant (oracle/talib_oracle.c; parity with TA-Lib itself is
    unpinned): rows sorted by (security, date), CSR ``offsets`` -> ``[n_rows][68]``."""
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    c = np.ascontiguousarray(close, dtype=np.float64)
    v = np.ascontiguousarray(volume, dtype=np.float64)
    n = int(offsets[-1])
    out = np.empty((n, TALIB_COLS), dtype=np.float64)
    longest = int(np.diff(offsets).max()) if len(offsets) > 1 else 0
    work = np.empty(4 * max(longest, 1), dtype=np.float64)
    lib().oracle_talib_panel(len(offsets) - 1, _p(offsets), _p(c), _p(v), _p(out), _p(work))
    return out

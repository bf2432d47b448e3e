"""Shared test helpers (synthetic panels -> oracle long arrays, bit-exact comparisons)."""
import numpy as np


def same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape:
        return False
    if a.dtype.kind == "f":
        return bool(((a == b) | (np.isnan(a) & np.isnan(b))).all())
    return bool((a == b).all())


def mismatch_report(a, b, names=None):
    bad = ~((a == b) | (np.isnan(a) & np.isnan(b)))
    if not bad.any():
        return "exact"
    cols = np.flatnonzero(bad.any(axis=0))
    msgs = []
    for j in cols[:8]:
        k = np.flatnonzero(bad[:, j])
        nm = names[j] if names is not None else j
        with np.errstate(all="ignore"):
            rel = np.nanmax(np.abs(a[k, j] - b[k, j]) / np.abs(b[k, j]))
        msgs.append(f"{nm}: {len(k)} cells, max rel {rel:.3g}, first row {k[0]}")
    return "; ".join(msgs)


def panel_long(p):
    """Synthetic Panel -> (t_idx, a_idx, offsets) of present cells in (asset, date) order."""
    v = p.valid[:, :p.A]
    aa, tt = np.nonzero(v.T)
    counts = v.sum(axis=0)
    offsets = np.r_[0, np.cumsum(counts)].astype(np.int64)
    return tt, aa, offsets


def oracle_panel(p):
    import oracle
    tt, aa, off = panel_long(p)
    fac = oracle.factors_long(off, p.close[tt, aa], p.volume[tt, aa], p.ret1d[tt, aa],
                              p.excess[tt, aa])
    return tt, aa, fac

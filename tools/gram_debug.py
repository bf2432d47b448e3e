#!/usr/bin/env python3
"""Debug helper: grid-mode Gram of a small synthetic panel vs numpy moments, per date; prints the
first dates whose count / means / centered moments disagree."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alpha-multi-factor-models_amd"))


def main(A=150, T=420, ncols=7):
    import torch
    import afm
    from afm.regression import xs_gram
    from afm.synthetic import make_panel
    grid = afm.PanelGrid.from_panel(make_panel(A, T, seed=21, tradable_p=0.9))
    out, nanfree = afm.factor_panel(grid)
    finite = afm.factor_panel(grid)[1]
    cols = list(range(ncols))
    ycol = 96
    lda = grid.lda
    gram, shift = xs_gram(out, T * lda, lda, grid.A, cols, ycol, bits=nanfree, nseg=T)
    G = gram.cpu().numpy()
    S = shift.cpu().numpy()
    O = out.cpu().numpy().reshape(98, T, lda)
    bits = nanfree.cpu().numpy().view(np.uint64)
    bad = 0
    for t in range(T):
        w = bits[t >> 6, :grid.A]
        m = ((w >> np.uint64(t & 63)) & np.uint64(1)).astype(bool)
        Z = np.stack([O[c, t, :grid.A] for c in cols + [ycol]], axis=1)[m]
        Z = Z[np.isfinite(Z).all(axis=1)]
        n = G[t, 0, 0]
        if n != len(Z) or (len(Z) and not np.all(np.isfinite(G[t]))):
            print(f"date {t}: n {n} vs {len(Z)}; finite gram {np.isfinite(G[t]).all()}; shift {S[t][:3]}")
            bad += 1
            if bad > 5:
                break
            continue
        if len(Z) == 0:
            continue
        mean = S[t, 1:] + G[t, 0, 1:] / n
        if not np.allclose(mean, Z.mean(axis=0), rtol=1e-11):
            print(f"date {t}: mean mismatch {np.abs(mean - Z.mean(0)).max()}")
            bad += 1
    print("bad dates:", bad)


if __name__ == "__main__":
    main()

"""Time afm_zgram_f64 (+ the tree merge) alone at config C, and check a few dates' Grams against a
torch fp64 reference of the same z-scored rows.  AFM_LIB selects a library variant (the
zgram experiments of the Makefile's `zgskip` target).

    python tools/zgram_probe.py [--assets 10000 --days 5040 --reps 5]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alpha-multi-factor-models_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--assets", type=int, default=10000)
    ap.add_argument("--days", type=int, default=5040)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--grid", type=int, default=0)
    ap.add_argument("--check", type=int, default=1)
    ap.add_argument("--chunks", type=str, default="16,32,64")
    a = ap.parse_args()
    import numpy as np
    import torch
    import afm
    from afm import _lib
    from afm.pipeline import Pipeline
    from afm.synthetic import make_panel
    p = make_panel(a.assets, a.days, seed=2023, tradable_p=0.9)
    grid = afm.PanelGrid.from_panel(p)
    pipe = Pipeline(grid)
    pipe.step()
    torch.cuda.synchronize()
    L, P = _lib.lib(), _lib.ptr
    T, lda = pipe.T, pipe.lda
    v1 = pipe.sp.v1
    h = pipe.ctx.bind_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    for nc in [int(x) for x in a.chunks.split(",")]:
        part = torch.empty((pipe.nrb, nc, pipe.pe), dtype=torch.float64, device=pipe.out.device)
        ts = []
        for _ in range(a.reps):
            ev[0].record()
            _lib.check(L.afm_zpool_f64(h, P(pipe.out), T * lda, lda, P(pipe.feat), None, pipe.p,
                                       96, P(pipe.zs), pipe.p, P(pipe.zrows), 0, v1, 0, pipe.nrb,
                                       pipe.A, nc, P(part), a.grid), "zpool")
            ev[1].record()
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]))
        print(f"zpool with {nc} chunks: {np.median(ts):.3f} ms (min {min(ts):.3f})", flush=True)
        del part
    tz, tm, tf = [], [], []
    for _ in range(a.reps):
        ev[0].record()
        _lib.check(L.afm_zpool_f64(h, P(pipe.out), T * lda, lda, P(pipe.feat), None, pipe.p, 96,
                                   P(pipe.zs), pipe.p, P(pipe.zrows), 0, v1, 0, pipe.nrb, pipe.A,
                                   64, P(pipe.pool_part), a.grid), "zpool")
        ev[1].record()
        pipe._pooled_blocks(h, 0, v1)
        ev[2].record()
        pipe._fm_local(h)
        ev[3].record()
        torch.cuda.synchronize()
        tz.append(ev[0].elapsed_time(ev[1]))
        tm.append(ev[1].elapsed_time(ev[2]))
        tf.append(ev[2].elapsed_time(ev[3]))
    rows = float(pipe.pool_g[0, 0, 0].item())
    p2 = pipe.p2
    tzm = float(np.median(tz))
    print(f"lib {os.environ.get('AFM_LIB', 'default')}: zpool {tzm:.3f} ms (min {min(tz):.3f}), "
          f"zpool+trees {np.median(tm):.3f} ms, fm (per-date grams + solve) {np.median(tf):.3f} "
          f"ms; rows {rows:.0f}; {rows * p2 * (p2 + 1) / tzm / 1e9:.2f} TF/s algorithmic",
          flush=True)
    if a.check and not os.environ.get("AFM_LIB"):
        from afm.grid import unpack_bits
        zr = unpack_bits(pipe.zrows, T)
        m = zr[:v1]
        tt, aa = torch.nonzero(m, as_tuple=True)
        X = pipe.out[pipe.feat.long()][:, tt, aa]                     # [p][n]
        Z = ((X - pipe.mu[:, aa]) / pipe.sd[:, aa]).T
        y = pipe.out[96][tt, aa]
        D = torch.cat([torch.ones_like(y)[:, None], Z, y[:, None]], dim=1)
        G = D.T @ D
        if pipe.sp.dup:                                   # train_end's rows count twice
            te = tt == pipe.sp.tr1 - 1
            G = G + D[te].T @ D[te]
        err = ((pipe.pool_g[0] - G).abs().max() / G.abs().max()).item()
        print(f"pooled gram vs torch fp64 reference: rel err {err:.3g}", flush=True)
        worst = 0.0
        fc = pipe.fm_cols.long()
        for t in np.linspace(300, T - 2, 6).astype(int):
            mm = zr[t]
            Z = pipe.out[fc, t][:, mm].T                              # raw FM columns
            y = pipe.out[96, t][mm]
            D = torch.cat([torch.ones_like(y)[:, None], Z, y[:, None]], dim=1)
            G = D.T @ D
            worst = max(worst, ((pipe.fm_gram[t] - G).abs().max() / G.abs().max()).item())
        print(f"FM per-date grams vs torch fp64 reference: worst rel err {worst:.3g}", flush=True)


if __name__ == "__main__":
    main()

"""Time the factor kernel alone at config C and print a checksum of its output planes and masks,
so build variants (AFM_LIB=<variant .so>) can be compared for speed and bit-identity.

    AFM_LIB=... python tools/fp_probe.py [--assets 10000 --days 5040 --reps 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alpha-multi-factor-models_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--assets", type=int, default=10000)
    ap.add_argument("--days", type=int, default=5040)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--listing-frac", type=float, default=0.1)
    ap.add_argument("--fast", type=int, default=1, help="context option factor_fast")
    ap.add_argument("--split", type=int, default=0, help="context option factor_split")
    a = ap.parse_args()
    import numpy as np
    import torch
    import afm
    from afm.synthetic import make_panel
    from afm import _lib
    grid = afm.PanelGrid.from_panel(make_panel(a.assets, a.days, seed=2023, tradable_p=0.9,
                                               listing_frac=a.listing_frac))
    _lib.Context.get().set_option("factor_fast", a.fast)
    _lib.Context.get().set_option("factor_split", a.split)
    out, nanfree = afm.factor_panel(grid)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(a.reps):
        ev[0].record()
        afm.factor_panel(grid, out=out, nanfree=nanfree)
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    bits = out.view(torch.int64)
    ck = [int(bits[i].sum()) & 0xffffffffffff for i in range(0, out.shape[0], 7)]
    ck.append(int(nanfree.sum()) & 0xffffffffffff)
    h = 0
    for v in ck:
        h = (h * 1000003 ^ v) & 0xffffffffffff
    # the label planes alone (afm_labels_f64, the side-stream kernel of the pipeline)
    L, P = _lib.lib(), _lib.ptr
    tl = []
    for _ in range(a.reps):
        ev[0].record()
        _lib.check(L.afm_labels_f64(_lib.Context.get().bind_stream(), grid.T, grid.lda, 0, grid.T,
                                    P(grid.excess), P(grid.ret1d), P(grid.vbits), P(out[96]),
                                    P(out[97])), "labels")
        ev[1].record()
        torch.cuda.synchronize()
        tl.append(ev[0].elapsed_time(ev[1]))
    print(f"labels alone {np.median(tl):.3f} ms", flush=True)
    print(f"lib={os.environ.get('AFM_LIB') or 'default'} A={a.assets} listing={a.listing_frac} "
          f"fast={a.fast} split={a.split}: factors {np.median(ts):.3f} ms "
          f"(min {min(ts):.3f}); checksum {h:012x}", flush=True)


if __name__ == "__main__":
    main()

"""Time afm_zscore_stats_f64 alone at config C (the pipeline's train-window statistics) and print a
hash of mu / sd, so variants (AFM_LIB=<experiment build>) can be compared for speed and bit-identity.

    AFM_LIB=<variant .so> python tools/zs_probe.py [--assets 10000 --days 5040 --reps 5]
"""
import argparse
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alpha-multi-factor-models_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--assets", type=int, default=10000)
    ap.add_argument("--days", type=int, default=5040)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    import torch
    import afm
    from afm import _lib
    from afm.pipeline import Pipeline
    from afm.synthetic import make_panel
    grid = afm.PanelGrid.from_panel(make_panel(a.assets, a.days, seed=2023, tradable_p=0.9))
    pipe = Pipeline(grid)
    pipe.step()
    torch.cuda.synchronize()
    L, P = _lib.lib(), _lib.ptr
    T, lda = pipe.T, pipe.lda_r
    h = pipe.ctx.bind_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(a.reps):
        ev[0].record()
        _lib.check(L.afm_zscore_stats_f64(h, P(pipe.out), T * lda, T, lda, P(pipe.feat), pipe.p,
                                          P(pipe.alldf), 0, pipe.sp.tr1, P(pipe.mu), P(pipe.sd)),
                   "zscore stats")
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    hsh = hashlib.sha1(pipe.mu.cpu().numpy().tobytes() + pipe.sd.cpu().numpy().tobytes()).hexdigest()
    print(f"lib={os.path.basename(os.path.dirname(os.environ.get('AFM_LIB') or 'afm/default'))}: zstats {np.median(ts):.3f} ms "
          f"(min {min(ts):.3f}); mu/sd sha1 {hsh[:16]}", flush=True)


if __name__ == "__main__":
    main()

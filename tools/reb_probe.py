"""Time afm_rebalance_f64 alone on the bench workload (pipeline state after one step) for the
AFM_REB_PROBE experiments: 0 full, 1 no QP, 2 no covariance, 3 neither.
    python tools/reb_probe.py [--top-n 100]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alpha-multi-factor-models_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--assets", type=int, default=10000)
    ap.add_argument("--days", type=int, default=5040)
    ap.add_argument("--top-n", type=int, default=100)
    a = ap.parse_args()
    import numpy as np
    import torch
    import afm
    from afm import _lib
    from afm.pipeline import Pipeline, PipelineConfig
    from afm.synthetic import make_panel
    p = make_panel(a.assets, a.days, seed=2023, tradable_p=0.9)
    grid = afm.PanelGrid.from_panel(p)
    pipe = Pipeline(grid, PipelineConfig(top_n=a.top_n))
    pipe.step()
    torch.cuda.synchronize()
    L, P = _lib.lib(), _lib.ptr
    c, full, x = pipe.cfg, pipe.full, pipe.reb_ext
    h = pipe.ctx.bind_stream()
    ne = pipe.e1 - pipe.e0
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for probe in os.environ.get("PROBES", "0,1,2,3,0").split(","):
        os.environ["AFM_REB_PROBE"] = probe
        ts = []
        for _ in range(3):
            ev[0].record()
            _lib.check(L.afm_rebalance_f64(h, pipe.T, full.A, full.lda, P(pipe.rd_ext), ne,
                                           P(pipe.pred), P(full.tbits), P(pipe.target),
                                           P(pipe.zrows_full), 0, pipe.sp.tr1, int(c.window),
                                           P(full.close), P(pipe.tmr), c.top_n, c.lo, c.hi,
                                           P(x["k"]), P(x["books"]), P(x["weights"]), P(x["sums"]),
                                           P(x["upos"]), P(x["usize"]), P(x["status"])), "reb")
            ev[1].record()
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]))
        print(f"top_n {a.top_n} probe {probe}: {np.median(ts):.3f} ms", flush=True)


if __name__ == "__main__":
    main()

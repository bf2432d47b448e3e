"""Time afm_min_variance_weights_f64 (one book: covariance + exact QP, one workgroup) for a few
book sizes -- the single-workgroup latency of the KKT path.
    python tools/qp_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alpha-multi-factor-models_amd")]


def main():
    import numpy as np
    import torch
    from afm import _lib
    ctx = _lib.Context.get(0)
    L, P = _lib.lib(), _lib.ptr
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for k in (10, 30, 64, 100, 128):
        rng = np.random.default_rng(k)
        rows = 252
        f = rng.normal(0, 0.01, (rows, 4))
        scale = rng.uniform(0.3, 2, k)
        scale[:3] = 0.05
        R = f @ rng.normal(0, 0.2, (4, k)) + rng.normal(0, 0.02, (rows, k)) * scale
        Rt = torch.as_tensor(R, device="cuda")
        w = torch.empty(k, dtype=torch.float64, device="cuda")
        cov = torch.empty((k, k), dtype=torch.float64, device="cuda")
        st = torch.empty(1, dtype=torch.int32, device="cuda")
        h = ctx.bind_stream()
        ts = []
        for _ in range(5):
            ev[0].record()
            _lib.check(L.afm_min_variance_weights_f64(h, P(Rt), rows, k, k, 0.0, 0.1, P(w), P(cov),
                                                      P(st)), "w")
            ev[1].record()
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]))
        print(f"k {k}: {np.median(ts) * 1e3:.1f} us (free {(w.cpu().numpy() > 1e-14).sum()})", flush=True)


if __name__ == "__main__":
    main()

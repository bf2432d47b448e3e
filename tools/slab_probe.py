#!/usr/bin/env python3
"""Config D pass time against the slab length (afm.intraday.factor_panel_slabs bars_per_slab).
    python tools/slab_probe.py 98304 65536 49152"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alpha-multi-factor-models_amd")]


def main():
    import torch
    from afm.intraday import factor_panel_slabs, make_panel_device, slab_bars
    g = make_panel_device(3000, 2 * 252 * 390, seed=2023)
    print("default slab", slab_bars(g), flush=True)
    for step in [int(s) for s in sys.argv[1:]]:
        times = []

        def consumer(t0, t1, out, nanfree):
            times.append(torch.cuda.Event(enable_timing=True))
            times[-1].record()
        factor_panel_slabs(g, lambda *x: None, step)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        t = time.perf_counter()
        n = factor_panel_slabs(g, consumer, step)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3
        per = [e0.elapsed_time(times[0])] + [times[i - 1].elapsed_time(times[i]) for i in range(1, n)]
        print(f"slab {step}: {n} slabs, pass {ms:.1f} ms, per slab " +
              " ".join(f"{x:.1f}" for x in per), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

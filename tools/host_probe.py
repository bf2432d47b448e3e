#!/usr/bin/env python3
"""Where does the HOST spend one Pipeline.step()?  Every libafm entry point is wrapped with a
timer (the ctypes call itself), and cProfile covers the Python / torch side.  A call that blocks
(an implicit device synchronisation) shows up as a long host time.

    python tools/host_probe.py [--assets 10000 --days 5040 --emulate-world 0 --steps 3]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alpha-multi-factor-models_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--assets", type=int, default=10000)
    ap.add_argument("--days", type=int, default=5040)
    ap.add_argument("--emulate-world", type=int, default=0)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import afm
    from afm import _lib
    from afm.pipeline import Pipeline, PipelineConfig
    from afm.synthetic import make_panel
    torch.cuda.set_device(0)
    grid = afm.PanelGrid.from_panel(make_panel(args.assets, args.days, seed=2023, tradable_p=0.9))
    comm = None
    if args.emulate_world > 1:
        from afm.sharded import EmulatedComm
        comm = EmulatedComm(args.emulate_world, 0)
    pipe = Pipeline(grid, PipelineConfig(), comm)
    for _ in range(2):
        pipe.step()
    torch.cuda.synchronize()

    lib = _lib.lib()
    host = defaultdict(float)
    count = defaultdict(int)
    orig = {}
    for name in _lib.SIGNATURES:
        if not name.startswith("afm_") or name in ("afm_last_error",):
            continue
        f = getattr(lib, name)
        orig[name] = f

        def wrap(*a, _f=f, _n=name):
            t = time.perf_counter()
            r = _f(*a)
            host[_n] += time.perf_counter() - t
            count[_n] += 1
            return r
        setattr(lib, name, wrap)

    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(args.steps):
        pipe.step()
    pr.disable()
    issued = time.perf_counter() - t0
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    for name, f in orig.items():
        setattr(lib, name, f)
    k = args.steps
    print(f"host issue {issued / k * 1e3:.3f} ms/step, wall {total / k * 1e3:.3f} ms/step")
    print("libafm calls by host time per step:")
    for n, v in sorted(host.items(), key=lambda x: -x[1])[:25]:
        print(f"  {n:34s} {v / k * 1e3:8.3f} ms  ({count[n] // k} calls)")
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()

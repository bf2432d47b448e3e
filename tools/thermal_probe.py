#!/usr/bin/env python3
"""Does a long GPU run slow the later bench lines down?  Times config D (bench.config_d_line)
cold, then after N headline steps, then again after a pause -- in one process.
    python tools/thermal_probe.py [--steps 400]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alpha-multi-factor-models_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    a = ap.parse_args()
    import torch
    import bench
    import afm
    from afm.pipeline import Pipeline, PipelineConfig
    from afm.synthetic import make_panel
    torch.cuda.set_device(0)
    d = bench.config_d_line(2023, 2)
    print(f"config D cold: {d['ms_per_pass']} ms", flush=True)
    grid = afm.PanelGrid.from_panel(make_panel(10000, 5040, seed=2023, tradable_p=0.9))
    pipe = Pipeline(grid, PipelineConfig())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        pipe.step()
        if k % 100 == 99:
            torch.cuda.synchronize()
            print(f"  steps {k + 1}: {(time.perf_counter() - t0) / (k + 1) * 1e3:.2f} ms/step", flush=True)
    del pipe, grid
    torch.cuda.empty_cache()
    d = bench.config_d_line(2023, 2)
    print(f"config D after {a.steps} headline steps: {d['ms_per_pass']} ms", flush=True)
    time.sleep(20)
    d = bench.config_d_line(2023, 2)
    print(f"config D after 20 s idle: {d['ms_per_pass']} ms", flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""A/B of PipelineConfig switches on the config-C step, each variant in its own process (one
Pipeline per process: two resident config-C pipelines slow the z-score and Gram stages), run in
alternation.  Usage: python tools/stage_ab.py [--steps 10 --rounds 2] [--lib-b PATH | --cfg-b JSON]
--lib-b: the same config on library variant B (AFM_LIB); --cfg-a / --cfg-b: two PipelineConfig
override sets (JSON); without either, the default build alone."""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alpha-multi-factor-models_amd")]


def child(cfgjson, steps):
    import numpy as np
    import torch
    import afm
    from afm.pipeline import PIPELINE_STAGES, Pipeline, PipelineConfig
    from afm.synthetic import make_panel
    grid = afm.PanelGrid.from_panel(make_panel(10000, 5040, seed=2023, tradable_p=0.9))
    pipe = Pipeline(grid, PipelineConfig(**json.loads(cfgjson)))
    for _ in range(2):
        pipe.step()
    evs = [{st: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            for st in PIPELINE_STAGES} for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        pipe.step(evs[i])
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    st = {s: float(np.mean([e[s][0].elapsed_time(e[s][1]) for e in evs])) for s in PIPELINE_STAGES}
    h = int(pipe.fm_beta.view(torch.int64).sum().item()) & 0xffffffffffff
    print(json.dumps({"ms": ms, "stages": st, "fm_hash": h, "lasso_hash":
                      int(pipe.lasso_beta.view(torch.int64).sum().item()) & 0xffffffffffff}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--lib-b", default=None)
    ap.add_argument("--cfg-a", default="{}", help="PipelineConfig overrides of A (JSON)")
    ap.add_argument("--cfg-b", default=None, help="PipelineConfig overrides of B (JSON)")
    ap.add_argument("--child", default=None)
    a = ap.parse_args()
    if a.child is not None:
        return child(a.child, a.steps)
    if a.cfg_b is not None:
        variants = {"A": (json.loads(a.cfg_a), None), "B": (json.loads(a.cfg_b), None)}
    elif a.lib_b:
        variants = {"A": ({}, None), "B": ({}, a.lib_b)}
    else:
        variants = {"default": ({}, None)}
    for _ in range(a.rounds):
        for name, (cfg, lib) in variants.items():
            env = dict(os.environ)
            if lib:
                env["AFM_LIB"] = lib
            r = subprocess.run([sys.executable, __file__, "--steps", str(a.steps), "--child",
                                json.dumps(cfg)], env=env, capture_output=True, text=True,
                               timeout=240)
            if r.returncode != 0:
                print(r.stderr[-2000:], flush=True)
                raise SystemExit(r.returncode)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            print(f"{name}: {d['ms']:.3f} ms/step  " +
                  " ".join(f"{s}={v:.2f}" for s, v in d["stages"].items()) +
                  f"  fm {d['fm_hash']:x} lasso {d['lasso_hash']:x}", flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-wave cycle profile of the factor kernel (needs the profiling build: make -C
alpha-multi-factor-models_amd prof; run with AFM_LIB=<that .so>)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alpha-multi-factor-models_amd"))


def main():
    import torch
    import afm
    from afm import _lib
    from afm.synthetic import make_panel
    A = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 5040
    torch.cuda.set_device(0)
    grid = afm.PanelGrid.from_panel(make_panel(A, T, seed=2023))
    afm.factor_panel(grid)
    torch.cuda.synchronize()
    L = _lib.lib()
    nblk = (A + 63) // 64
    # AFM_FP_TYPES: the launch code the run used (factor_split; 1xx = the 30-set partition with
    # xx workgroups per block, 2xx = the 60-set one)
    code = int(os.environ.get('AFM_FP_TYPES', '3'))
    if code > 200:
        types, jw = code - 200, 60 // (code - 200)
    elif code > 100:
        types, jw = code - 100, 30 // (code - 100)
    else:
        types, jw = code, 15 // code
    if code:
        _lib.Context.get().set_option("factor_split", code)
        afm.factor_panel(grid)
        torch.cuda.synchronize()
    n = nblk * types * jw * 4
    buf = (ctypes.c_longlong * n)()
    assert L.afm_debug_wave_cycles(buf, n) == 0
    c = np.frombuffer(buf, dtype=np.int64).reshape(nblk, types, jw, 4)
    tot, wait = c[..., 0] / 1e6, c[..., 1] / 1e6
    print("Mcycles per wave (mean over blocks): total | barrier wait")
    for t in range(types):
        print(f"type {t}: " + "  ".join(f"w{w} {tot[:, t, w].mean():7.2f}|{wait[:, t, w].mean():6.2f}"
                                        for w in range(jw)))
    st = (c[..., 2] - c[..., 2].min()) / 1e2
    print("workgroup start (us after the first, 100 MHz clock): percentiles 0/25/50/75/90/100:",
          np.percentile(st[:, :, 0], [0, 25, 50, 75, 90, 100]).round(2))
    dt = (c[..., 3] - c[..., 2]) * 1e-8                      # seconds (100 MHz clock)
    print(f"shader clock estimate: {np.median(c[..., 0] / dt) / 1e9:.3f} GHz (cycles / real time)")
    print(f"max total {tot.max():.2f} Mcycles; per type max: "
          + " ".join(f"{tot[:, t].max():.2f}" for t in range(types)))


if __name__ == "__main__":
    main()

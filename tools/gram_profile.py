#!/usr/bin/env python3
"""Per-wave cycle profile of the Gram kernel (profiling build: make -C alpha-multi-factor-models_amd
prof; run with AFM_LIB=<that .so>): total loop cycles and barrier-wait cycles of the consumer
(MFMA) and producer waves, over the first 4096 dates' workgroups."""
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
    from afm.pipeline import Pipeline
    from afm.synthetic import make_panel
    torch.cuda.set_device(0)
    grid = afm.PanelGrid.from_panel(make_panel(10000, 5040, seed=2023))
    pipe = Pipeline(grid)
    pipe.step()
    torch.cuda.synchronize()
    n = 4096 * 8 * 2
    buf = (ctypes.c_longlong * n)()
    assert _lib.lib().afm_debug_gram_cycles(buf, n) == 0
    c = np.frombuffer(buf, dtype=np.int64).reshape(4096, 8, 2)[1000:4000] / 1e3
    for w in range(8):
        role = "consumer" if w < 4 else "producer"
        print(f"wave {w} ({role}): total {c[:, w, 0].mean():8.1f} kcycles, barrier wait "
              f"{c[:, w, 1].mean():8.1f} kcycles")


if __name__ == "__main__":
    main()

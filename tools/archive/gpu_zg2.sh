#!/bin/bash
# zpool priority A/B (AFM_ZG_PRIO 1: producers high (default), 0: equal, 2: consumers high)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for pr in 1 0 2 3; do
  AFM_ZG_PRIO=$pr timeout -k 10 200 python -u tools/zgram_probe.py --check 0 > gpurun_out/zg_prio$pr.log 2>&1 || { cat gpurun_out/zg_prio$pr.log; exit 1; }
  echo "prio $pr: $(grep zpool gpurun_out/zg_prio$pr.log)"
done

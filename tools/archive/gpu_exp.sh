#!/bin/bash
# Kernel A/B experiments (box): the z-statistics load batch (AFM_ZS_U), each variant in its own
# process (the choice is read once), timed alone at config C with a hash of its results.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for u in ${ZS_VARIANTS:-8 16 32}; do
  AFM_ZS_U=$u timeout -k 10 240 python -u tools/zs_probe.py > gpurun_out/exp_zs$u.log 2>&1 || { tail -20 gpurun_out/exp_zs$u.log; exit 1; }
  grep zstats gpurun_out/exp_zs$u.log
done

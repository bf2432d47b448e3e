#!/bin/bash
# Factor kernel at per-rank shard sizes (box): assets x split override (AFM_FP_TYPES)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for A in ${FP_ASSETS:-10000 5000 2500 1250}; do for t in ${FP_TYPES_LIST:-3 5 15}; do
  AFM_FP_TYPES=$t timeout -k 10 120 python -u tools/fp_probe.py --assets $A > gpurun_out/fps_${A}_$t.log 2>&1 || { tail -5 gpurun_out/fps_${A}_$t.log; exit 1; }
  echo "assets $A types $t: $(grep -o 'factors [0-9.]* ms (min [0-9.]*)' gpurun_out/fps_${A}_$t.log)"
done; done

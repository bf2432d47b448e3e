#!/bin/bash
# factor kernel A/B over shard sizes: base (round 2), 15-set, 21-set; 3 alternating rounds
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/fpab3; o=gpurun_out/fpab3
for A in 10000 2500 1250; do
  for round in 1 2 3; do
    for lib in alpha-multi-factor-models_amd/build/exp/base/libafm.so default alpha-multi-factor-models_amd/build/exp/fp21/libafm.so; do
      if [ "$lib" = default ]; then L=""; else L=$R/$lib; fi
      AFM_LIB=$L timeout -k 10 120 python -u tools/fp_probe.py --assets $A --reps 7 2>&1 | grep "factors" | sed "s|$R/||" || exit 1
    done
  done
done

#!/bin/bash
# factor kernel decomposition: store-pattern probe, no-store variants, A/B
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/fpx2; o=gpurun_out/fpx2
for m in 0 1 2 4 5; do timeout -k 10 60 tools/store_probe/store_probe 5040 10000 $m | tail -2; done
for lib in default alpha-multi-factor-models_amd/build/exp/nostore/libafm.so alpha-multi-factor-models_amd/build/exp/nostore21/libafm.so; do
  if [ "$lib" = default ]; then L=""; else L=$R/$lib; fi
  AFM_LIB=$L timeout -k 10 200 python -u tools/fp_probe.py --reps 5 2>&1 | grep factors
done

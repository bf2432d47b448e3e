#!/bin/bash
# Lasso alone on the dense-variant and headline Grams: product vs the round-3 kernel (l3)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4m; mkdir -p $o
P=$R/alpha-multi-factor-models_amd/build/exp
for lib in default $P/l3/libafm.so default; do
  if [ "$lib" = default ]; then L=""; else L=$lib; fi
  AFM_LIB=$L timeout -k 10 200 python -u tools/lasso_probe.py 10000 5 2>&1 | grep lasso | tee -a $o/lasso.txt || exit 1
done

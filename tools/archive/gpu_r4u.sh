#!/bin/bash
# xs_stats time split (timing-only: skip1 = no Welford lanes, skip2 = no layer lanes)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4u; mkdir -p $o
P=$R/alpha-multi-factor-models_amd/build/exp
for lib in $P/skip1/libafm.so $P/skip2/libafm.so; do
  if [ "$lib" = default ]; then L=""; else L=$lib; fi
  echo "== $lib" | tee -a $o/an.txt
  AFM_LIB=$L timeout -k 10 200 python -u tools/an_probe.py 2>&1 | grep -E "xs_stats" | grep -v outputs | tee -a $o/an.txt || exit 1
done

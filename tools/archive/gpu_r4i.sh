#!/bin/bash
# A/B: factor job partitions (current / light-heavy p2 / p3), parity of p3, per-wave profiles
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4i; mkdir -p $o
P=$R/alpha-multi-factor-models_amd/build/exp
AFM_LIB=$P/p3/libafm.so timeout -k 10 300 python -u -m pytest tests/test_factors_gpu.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
for lib in default $P/p2/libafm.so $P/p3/libafm.so; do
  if [ "$lib" = default ]; then L=""; else L=$lib; fi
  for A in 10000 1250; do
    echo "$lib" >> $o/fp.txt
    AFM_LIB=$L timeout -k 10 200 python -u tools/fp_probe.py --assets $A --reps 5 2>&1 | grep factors | tee -a $o/fp.txt || exit 1
  done
done
done
for v in p1prof p3prof; do
  AFM_LIB=$P/$v/libafm.so timeout -k 10 200 python -u tools/wave_profile.py > $o/wave_$v.txt 2>&1 || { tail -5 $o/wave_$v.txt; exit 1; }
  cat $o/wave_$v.txt
done

#!/bin/bash
# factor partition: SMA_6 moved from W9 to W2 (variant mv) vs product; factor / intraday tests on mv
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4x2; mkdir -p $o
P=$R/alpha-multi-factor-models_amd/build/exp
AFM_LIB=$P/mv/libafm.so timeout -k 10 300 python -u -m pytest tests/test_factors_gpu.py tests/test_intraday_gpu.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head; exit 1; }
for r in 1 2; do
for lib in default $P/mv/libafm.so; do
  if [ "$lib" = default ]; then L=""; else L=$lib; fi
  for A in 1250 2500 10000; do
    echo "$lib" >> $o/fp.txt
    AFM_LIB=$L timeout -k 10 200 python -u tools/fp_probe.py --assets $A --reps 5 2>&1 | grep factors | tee -a $o/fp.txt || exit 1
  done
done
done

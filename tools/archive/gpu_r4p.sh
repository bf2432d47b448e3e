#!/bin/bash
# Lasso coordinate loop A/B: product vs variant l7 (the likely next coordinate's LDS data read ahead)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4p; mkdir -p $o
P=$R/alpha-multi-factor-models_amd/build/exp
AFM_LIB=$P/l7/libafm.so timeout -k 10 300 python -u -m pytest tests/test_lasso.py -x -q -m gpu --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head; exit 1; }
for lib in default $P/l7/libafm.so default $P/l7/libafm.so; do
  if [ "$lib" = default ]; then L=""; else L=$lib; fi
  AFM_LIB=$L timeout -k 10 200 python -u tools/lasso_probe.py 10000 5 2>&1 | grep lasso | tee -a $o/lasso.txt || exit 1
done

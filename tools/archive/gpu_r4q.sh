#!/bin/bash
# PnL scan: two-level dataflow on loader-derived grandchildren (product) vs one level (pbase); portfolio / chain / config tests
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4q; mkdir -p $o
P=$R/alpha-multi-factor-models_amd/build/exp
timeout -k 10 600 python -u -m pytest tests/test_portfolio_gpu.py tests/test_chain_gpu.py tests/test_configs_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -20; exit 1; }
for lib in $P/pbase/libafm.so default $P/pbase/libafm.so default; do
  if [ "$lib" = default ]; then L=""; else L=$lib; fi
  AFM_LIB=$L timeout -k 10 200 python -u tools/pnl_probe.py --reps 20 2>&1 | grep -E "afm_pnl|value" | tee -a $o/pnl.txt || exit 1
done

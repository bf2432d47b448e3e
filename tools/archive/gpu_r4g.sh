#!/bin/bash
# A/B: factor kernel chunk hand-off (barrier 8-day / counters 8-day / counters 4-day); PnL dataflow
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4g; mkdir -p $o
P=$R/alpha-multi-factor-models_amd/build/exp
timeout -k 10 400 python -u -m pytest tests/test_portfolio_gpu.py tests/test_chain_gpu.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/pnl_probe.py > $o/pnl.txt 2>&1 || { tail -5 $o/pnl.txt; exit 1; }
grep afm_pnl $o/pnl.txt
for r in 1 2; do
for lib in default $P/bar8/libafm.so $P/cnt8/libafm.so; do
  if [ "$lib" = default ]; then L=""; else L=$lib; fi
  for A in 10000 1250; do
    AFM_LIB=$L timeout -k 10 200 python -u tools/fp_probe.py --assets $A --reps 5 2>&1 | grep factors | tee -a $o/fp.txt || exit 1
  done
done
done

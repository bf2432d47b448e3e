#!/bin/bash
# two-day pipelined fast steps in the split launches (small panels): parity + A/B + profile
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4k; mkdir -p $o
P=$R/alpha-multi-factor-models_amd/build
timeout -k 10 300 python -u -m pytest tests/test_factors_gpu.py tests/test_intraday_gpu.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head; exit 1; }
for r in 1 2; do
for lib in default $P/exp/base/libafm.so; do
  if [ "$lib" = default ]; then L=""; else L=$lib; fi
  for A in 1250 2500 10000; do
    echo "$lib" >> $o/fp.txt
    AFM_LIB=$L timeout -k 10 200 python -u tools/fp_probe.py --assets $A --reps 5 2>&1 | grep factors | tee -a $o/fp.txt || exit 1
  done
done
done
AFM_FP_TYPES=15 AFM_LIB=$P/prof/libafm.so timeout -k 10 200 python -u tools/wave_profile.py 1250 > $o/wave1250.txt 2>&1 || { tail -5 $o/wave1250.txt; exit 1; }
cat $o/wave1250.txt

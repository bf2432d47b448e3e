#!/bin/bash
# round 5: software-pipelined clean steps in the 30-set partition -- factor parity, then A/B factor
# times (product vs build/exp/nofuse = the previous product) at shard / config sizes
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5f; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_factors_gpu.py tests/test_intraday_gpu.py -x -v --timeout 300 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -30; exit 1; }
for rep in 1 2; do
for A in 1250 3000 5000; do
  timeout -k 10 120 python -u tools/fp_probe.py --assets $A --reps 5 >> $o/fp.txt 2>&1 || { tail -5 $o/fp.txt; exit 1; }
  AFM_LIB=$R/alpha-multi-factor-models_amd/build/exp/nofuse/libafm.so timeout -k 10 120 python -u tools/fp_probe.py --assets $A --reps 5 >> $o/fp.txt 2>&1 || { tail -5 $o/fp.txt; exit 1; }
done
done
timeout -k 10 120 python -u tools/fp_probe.py --assets 10000 --reps 5 >> $o/fp.txt 2>&1 || { tail -5 $o/fp.txt; exit 1; }
grep factors $o/fp.txt

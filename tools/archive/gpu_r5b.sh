#!/bin/bash
# round 5: the 30-set small-grid factor partition -- factor / intraday parity, then factor times
# and checksums at shard / config sizes (auto launch shape and forced PartC)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5b; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_factors_gpu.py tests/test_intraday_gpu.py -x -v --timeout 300 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -30; exit 1; }
for A in 1250 2500 3000 5000 10000; do
  timeout -k 10 120 python -u tools/fp_probe.py --assets $A --reps 5 >> $o/fp.txt 2>&1 || { tail -5 $o/fp.txt; exit 1; }
done
for A in 1250 3000; do
  timeout -k 10 120 python -u tools/fp_probe.py --assets $A --reps 5 --split 15 >> $o/fp.txt 2>&1 || { tail -5 $o/fp.txt; exit 1; }
done
cat $o/fp.txt | grep factors

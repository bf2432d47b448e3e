#!/bin/bash
# round 5: PartS next-observation prefetch (product) and static LDS (build/exp/stat) vs the previous
# product (build/exp/nofuse): factor parity, then factor times / checksums at shard sizes
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5j; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_factors_gpu.py tests/test_intraday_gpu.py -x -v --timeout 300 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -30; exit 1; }
for rep in 1 2; do
for A in 1250 3000 5000; do
  for L in default stat nofuse; do
    if [ $L = default ]; then unset AFM_LIB; else export AFM_LIB=$R/alpha-multi-factor-models_amd/build/exp/$L/libafm.so; fi
    timeout -k 10 120 python -u tools/fp_probe.py --assets $A --reps 5 >> $o/fp.txt 2>&1 || { tail -5 $o/fp.txt; exit 1; }
  done
  unset AFM_LIB
done
done
grep factors $o/fp.txt

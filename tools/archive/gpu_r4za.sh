#!/bin/bash
# z statistics with the reciprocal-table Welford quotient (variant za: every row of a full 8-date block read, presence bit tested with the NaN check) vs product: zscore / chain /
# sharded tests on zt, zs_probe speed + mu/sd hash A/B, headline bench A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4za; mkdir -p $o
Z=$R/alpha-multi-factor-models_amd/build/exp/za/libafm.so
AFM_LIB=$Z timeout -k 10 400 python -u -m pytest tests/test_zscore_gpu.py tests/test_chain_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head; exit 1; }
for r in 1 2; do
  for L in "" $Z; do
    AFM_LIB=$L timeout -k 10 200 python -u tools/zs_probe.py --reps 7 2>&1 | grep zstats | tee -a $o/zs.txt || exit 1
  done
done
for r in 1 2; do
  for L in "" $Z; do
    echo "lib=${L:-default}" >> $o/bench.txt
    AFM_LIB=$L timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-variants 2>/dev/null | tail -1 | tee -a $o/bench.txt || exit 1
  done
done

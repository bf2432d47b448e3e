#!/bin/bash
# z statistics with the reciprocal-table Welford quotient (variant zt) vs product: zscore / chain /
# sharded tests on zt, zs_probe speed + mu/sd hash A/B, headline bench A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4zt; mkdir -p $o
Z=$R/alpha-multi-factor-models_amd/build/exp/zt/libafm.so
AFM_LIB=$Z timeout -k 10 400 python -u -m pytest tests/test_zscore_gpu.py tests/test_chain_gpu.py tests/test_sharded.py -x -q -m gpu --timeout 200 --timeout-method thread > $o/tests.log 2>&1
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

#!/bin/bash
# round 5: the 60-set factor partition PartT (codes 212 / 210 / 206) -- bit-exactness of every
# split, slab carry, sharded / chain parity; then fp_probe PartT vs PartS at shard sizes
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5r; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_factors_gpu.py tests/test_intraday_gpu.py tests/test_sharded.py tests/test_chain_gpu.py -x -v -m gpu --timeout 400 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -30; exit 1; }
for A in 1250 2500 1600 640; do
  for sp in 0 110 106 103; do
    timeout -k 10 200 python -u tools/fp_probe.py --assets $A --listing-frac 0.1 --reps 5 --split $sp > $o/fp_${A}_$sp.txt 2>&1 || { echo "fp $A $sp failed"; tail -5 $o/fp_${A}_$sp.txt; exit 1; }
    tail -1 $o/fp_${A}_$sp.txt
  done
done

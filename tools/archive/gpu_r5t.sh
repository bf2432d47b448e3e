#!/bin/bash
# round 5: loader with three chunks of loads in flight + unrolled combiners -- parity of every
# split / slab / sharded / chain test, then fp_probe across sizes and partitions
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5t; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_factors_gpu.py tests/test_intraday_gpu.py tests/test_sharded.py tests/test_chain_gpu.py -x -v -m gpu --timeout 400 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -30; exit 1; }
for cfg in "1250 0" "1250 110" "1250 210" "1250 206" "2500 0" "2500 106" "2500 206" "3000 0" "3000 206" "10000 0"; do
  set -- $cfg
  timeout -k 10 200 python -u tools/fp_probe.py --assets $1 --listing-frac 0.1 --reps 5 --split $2 > $o/fp_$1_$2.txt 2>&1 || { echo "fp $cfg failed"; tail -5 $o/fp_$1_$2.txt; exit 1; }
  tail -1 $o/fp_$1_$2.txt
done

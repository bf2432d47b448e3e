#!/bin/bash
# xs_stats: batched staging loads + 8-row Welford blocks with the next block's LDS reads in flight (product) vs an0 (HEAD)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4t; mkdir -p $o
P=$R/alpha-multi-factor-models_amd/build/exp
timeout -k 10 600 python -u -m pytest tests/test_analyzer_gpu.py tests/test_chain_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -20; exit 1; }
for lib in $P/an0/libafm.so default $P/an0/libafm.so default; do
  if [ "$lib" = default ]; then L=""; else L=$lib; fi
  echo "== $lib" >> $o/an.txt
  AFM_LIB=$L timeout -k 10 200 python -u tools/an_probe.py 2>&1 | grep -E "xs_stats|lib=" | tee -a $o/an.txt || exit 1
done

#!/bin/bash
# analyzer on the CUs the CU-masked FM stream leaves free (B) vs default placement (A)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4w; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_chain_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -20; exit 1; }
for k in 32 64 16; do
  echo "== fm_free_cus $k + analyzer_free_cus" | tee -a $o/ab.txt
  timeout -k 10 900 python -u tools/stage_ab.py --steps 10 --rounds 2 --cfg-a '{}' --cfg-b "{\"fm_free_cus\": $k, \"analyzer_free_cus\": true}" 2>&1 | tee -a $o/ab.txt || exit 1
done

#!/bin/bash
# FM Grams forked after the analyzer's xs_prepare (B) vs after the predict (A)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4s; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_chain_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -20; exit 1; }
timeout -k 10 900 python -u tools/stage_ab.py --steps 10 --rounds 3 --cfg-a '{}' --cfg-b '{"fm_fork": "prepare"}' 2>&1 | tee $o/ab.txt || exit 1

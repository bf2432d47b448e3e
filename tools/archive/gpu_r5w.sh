#!/bin/bash
# round 5: factor / intraday parity after trimming PartT to code 206; PMC traffic of the headline
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5w; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_factors_gpu.py tests/test_intraday_gpu.py -x -q -m gpu --timeout 400 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -30; exit 1; }
bash tools/gpu_pmc.sh r5w

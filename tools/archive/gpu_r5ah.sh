#!/bin/bash
# round 5: pipelined Lasso coordinate loop -- parity and the dense-variant timing
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5ah; mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lasso.py tests/test_chain_gpu.py > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 300 python -u tools/lasso_probe.py 10000 5 > $o/probe.log 2>&1 || { tail -20 $o/probe.log; exit 1; }
grep lib= $o/probe.log

#!/bin/bash
# round 5: the dense-variant Lasso alone; save its Gram for the CPU analysis of the sweep
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5ag; mkdir -p $o
LASSO_SAVE=$o timeout -k 10 300 python -u tools/lasso_probe.py 10000 5 > $o/probe.log 2>&1 || { tail -20 $o/probe.log; exit 1; }
cat $o/probe.log

#!/bin/bash
# QP / rebalance check: the portfolio GPU tests, then the rebalance alone at top_n = 100 by phase.
# Usage (box): tools/gpu_qp.sh <tag>
TAG=$1
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_portfolio_gpu.py -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 \
    || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
AFM_LIB=alpha-multi-factor-models_amd/build/prof/libafm.so PROBES=0,1,4 timeout -k 10 300 python -u tools/reb_probe.py --top-n 100 > gpurun_out/${TAG}_reb.log 2>&1 \
    || { echo "probe failed"; tail -20 gpurun_out/${TAG}_reb.log; exit 1; }
grep -v Warn gpurun_out/${TAG}_reb.log | grep -v amdgpu.ids

#!/bin/bash
# round 5: one-wave turnover DAG records + small-chunk PnL scan for bootstrap paths -- parity
# (portfolio, chain, configs, sharded), then the config E line and its kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5l; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_portfolio_gpu.py tests/test_chain_gpu.py tests/test_configs_gpu.py tests/test_sharded.py -x -v -m gpu --timeout 400 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -30; exit 1; }
timeout -k 10 300 python -u bench.py --config-only e > $o/e.json 2> $o/e.err || { tail -5 $o/e.err; exit 1; }
cat $o/e.json | cut -c1-700
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5l_e -o run --output-format csv -- \
    python3 $R/bench.py --config-only e > $R/gpurun_out/r5l_e.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/r5l_e.log; exit 1; }
cd $R; python3 tools/rocprof_summary.py gpurun_out/r5l_e/run_kernel_trace.csv > gpurun_out/r5l_e_kernel_stats.txt; head -14 gpurun_out/r5l_e_kernel_stats.txt

#!/bin/bash
# Pooled Gram (box): chain + sharded + regression GPU tests, then the zpool timing.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_chain_gpu.py tests/test_sharded.py tests/test_regression_gpu.py tests/test_configs_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/zp_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/zp_tests.log | tail -24
[ $rc -ne 0 ] && { tail -40 gpurun_out/zp_tests.log; exit $rc; }
timeout -k 10 240 python -u tools/zgram_probe.py --check 1 --chunks 64 > gpurun_out/zp.log 2>&1 || { tail -20 gpurun_out/zp.log; exit 1; }
grep -E 'zpool|rel err' gpurun_out/zp.log

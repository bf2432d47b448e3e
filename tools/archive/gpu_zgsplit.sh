#!/bin/bash
# pooled Gram: half-pair split variant vs default (time + fp64 check), then the Gram-dependent GPU
# tests on the variant
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/zgsplit; mkdir -p $o
V=$R/alpha-multi-factor-models_amd/build/exp/zgsplit/libafm.so
for round in 1 2; do
  timeout -k 10 200 python -u tools/zgram_probe.py --check 0 2>&1 | grep "^lib" || exit 1
  AFM_LIB=$V timeout -k 10 200 python -u tools/zgram_probe.py --check 0 2>&1 | grep "^lib" || exit 1
done
AFM_LIB=$V timeout -k 10 500 python -u -m pytest tests/test_zgram_wide_gpu.py tests/test_chain_gpu.py tests/test_configs_gpu.py \
   tests/test_sharded.py tests/test_regression_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $o/tests.log 2>&1 \
   || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log

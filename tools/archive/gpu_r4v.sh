#!/bin/bash
# pooled Gram: 16-B staging producer (variant zw) vs product; Gram / chain / sharded tests on zw
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4v; mkdir -p $o
P=$R/alpha-multi-factor-models_amd/build/exp
AFM_LIB=$P/zw/libafm.so timeout -k 10 600 python -u -m pytest tests/test_zgram_wide_gpu.py tests/test_configs_gpu.py tests/test_chain_gpu.py tests/test_sharded.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -20; exit 1; }
timeout -k 10 900 python -u tools/stage_ab.py --steps 10 --rounds 3 --lib-b $P/zw/libafm.so 2>&1 | tee $o/ab.txt || exit 1

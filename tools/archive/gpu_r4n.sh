#!/bin/bash
# early z statistics (two factor slabs): chain placement + sharded bit-identity tests, per-rank proxy
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4n; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_chain_gpu.py tests/test_sharded.py tests/test_factors_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -20; exit 1; }
for w in 8 4; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --emulate-world $w > $o/emu$w.json 2> $o/emu$w.err || { tail -5 $o/emu$w.err; exit 1; }
  cat $o/emu$w.json
done

#!/bin/bash
# z statistics launch by grid fill (1,024-thread workgroups only when they fill the chip): zscore /
# chain / sharded tests, zs_probe at config C and the N = 8 shard, emulated N = 8 proxy
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4zw; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_zscore_gpu.py tests/test_chain_gpu.py tests/test_sharded.py -x -q -m gpu --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head; exit 1; }
for A in 10000 1250; do
  timeout -k 10 200 python -u tools/zs_probe.py --assets $A --reps 7 2>&1 | grep zstats | sed "s/^/A=$A /" | tee -a $o/zs.txt || exit 1
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --emulate-world 8 2>/dev/null | tail -1 | tee $o/emu8.json || exit 1

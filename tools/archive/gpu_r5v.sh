#!/bin/bash
# round 5: the exchanges' placement copies batched (one reorder + one copy per plane, one
# index_select per rebalance key) -- sharded parity, then the emulated rank steps
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5v; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_sharded.py tests/test_configs_gpu.py -x -v -m gpu --timeout 400 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -30; exit 1; }
for w in 8 4 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --emulate-world $w > $o/emu$w.json 2> $o/emu$w.err || { tail -5 $o/emu$w.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$o/emu$w.json').read().strip().splitlines()[-1])
print('emu$w', d['ms_per_step'], {k: round(v,2) for k,v in d.get('stage_ms',{}).items()})"
done

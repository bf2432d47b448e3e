#!/bin/bash
# round 5: exchange placement without intermediate copies (_place one strided copy, packed-gather
# views) -- sharded / chain GPU tests and the emulated rank steps
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5ak; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sharded.py tests/test_chain_gpu.py > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for rep in 1 2; do
for w in 8 4; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --emulate-world $w > $o/emu$w.$rep.json 2> $o/emu$w.$rep.err || { tail -5 $o/emu$w.$rep.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$o/emu$w.$rep.json').read().strip().splitlines()[-1])
print('emu$w', d['ms_per_step'], {k: round(v,2) for k,v in d.get('stage_ms',{}).items()})"
done
done

#!/bin/bash
# round 5: streamed z statistics with the train window split into the slabs and the post-train
# dates in one (the last statistics slab beside the post-train factor slab) vs even slabs
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5al; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_chain_gpu.py tests/test_zscore_gpu.py tests/test_sharded.py > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for rep in 1 2; do
for v in split even; do
  f=""; [ $v = even ] && f="--zstats-even"
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --emulate-world 8 $f > $o/emu8_$v.$rep.json 2> $o/emu8_$v.$rep.err || { tail -5 $o/emu8_$v.$rep.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$o/emu8_$v.$rep.json').read().strip().splitlines()[-1])
print('emu8 $v $rep', d['ms_per_step'], {k: round(v,2) for k,v in d.get('stage_ms',{}).items()})"
done
done

#!/bin/bash
# round 5: streamed z statistics -- slab count A/B on the emulated world-8 rank step
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5z2; mkdir -p $o
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1])
print('$2', d['ms_per_step'], {k: round(v,2) for k,v in d.get('stage_ms',{}).items()})"; }
for rep in 1 2; do
  for S in 0 4 6 8; do
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --emulate-world 8 --zstats-slabs $S --no-cpu-baseline --no-configs --no-variants > $o/emu8_$S.$rep.json 2> $o/emu8_$S.$rep.err || { echo "S=$S failed"; tail -5 $o/emu8_$S.$rep.err; exit 1; }
    show $o/emu8_$S.$rep.json "emu8 S=$S $rep"
  done
done
timeout -k 10 900 python -u -m pytest tests/test_chain_gpu.py tests/test_sharded.py -x -q -m gpu --timeout 400 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -30; exit 1; }

#!/bin/bash
# round 5: small-grid z statistics with two columns per thread -- parity, then the emulated
# world-8 / 4 rank steps and config B against one column per thread (nc1)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5y; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_zscore_gpu.py tests/test_sharded.py tests/test_chain_gpu.py -x -q -m gpu --timeout 400 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -30; exit 1; }
B=alpha-multi-factor-models_amd/build/exp
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1])
print('$2', d['ms_per_step'], {k: round(v,2) for k,v in d.get('stage_ms',{}).items()})"; }
for rep in 1 2; do
  for v in default nc1; do
    if [ $v = default ]; then lib=""; else lib=$R/$B/$v/libafm.so; fi
    for w in 8 4; do
      AFM_LIB=$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --emulate-world $w --no-cpu-baseline --no-configs --no-variants > $o/emu${w}_$v.$rep.json 2> $o/emu${w}_$v.$rep.err || { echo "emu$w $v failed"; tail -5 $o/emu${w}_$v.$rep.err; exit 1; }
      show $o/emu${w}_$v.$rep.json "emu$w $v $rep"
    done
    AFM_LIB=$lib timeout -k 10 300 python -u bench.py --config-only b > $o/b_$v.$rep.json 2> $o/b_$v.$rep.err || { echo "b $v failed"; tail -5 $o/b_$v.$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$o/b_$v.$rep.json').read().strip().splitlines()[-1])['config_b']
print('B $v $rep', d['ms_per_step'], d['stage_ms'])"
  done
done

#!/bin/bash
# round 5: the streamed z-statistics slab kernel with Markstein quotients from reciprocals
# computed ahead of the chain -- parity, then the emulated N = 8 step against the IEEE-division
# slab kernel (zsdiv)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5ab; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_zscore_gpu.py tests/test_chain_gpu.py tests/test_sharded.py -x -q -m gpu --timeout 400 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -30; exit 1; }
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1])
print('$2', d['ms_per_step'], {k: round(v,2) for k,v in d.get('stage_ms',{}).items()})"; }
B=alpha-multi-factor-models_amd/build/exp
for rep in 1 2; do
  for v in default zsdiv; do
    if [ $v = default ]; then lib=""; else lib=$R/$B/$v/libafm.so; fi
    AFM_LIB=$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --emulate-world 8 --no-cpu-baseline --no-configs --no-variants > $o/emu8_$v.$rep.json 2> $o/emu8_$v.$rep.err || { echo "$v failed"; tail -5 $o/emu8_$v.$rep.err; exit 1; }
    show $o/emu8_$v.$rep.json "emu8 $v $rep"
  done
done

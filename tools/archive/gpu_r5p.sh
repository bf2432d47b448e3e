#!/bin/bash
# round 5: priority split A/B (tail kernels T, PnL scan + turnover records S) on the headline and
# the emulated world-8 rank step; portfolio / chain / sharded parity first
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5p; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_portfolio_gpu.py tests/test_chain_gpu.py tests/test_sharded.py tests/test_zgram_wide_gpu.py tests/test_zscore_gpu.py -x -v -m gpu --timeout 400 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -30; exit 1; }
B=alpha-multi-factor-models_amd/build/exp
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1])
print('$2', d['ms_per_step'], {k: round(v,2) for k,v in d.get('stage_ms',{}).items()})"; }
for rep in 1 2; do
  for v in default t2s3 t1s3 t3s0; do
    if [ $v = default ]; then lib=""; else lib=$R/$B/$v/libafm.so; fi
    AFM_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-configs --no-variants > $o/$v.$rep.json 2> $o/$v.$rep.err || { echo "$v failed"; tail -5 $o/$v.$rep.err; exit 1; }
    show $o/$v.$rep.json "$v $rep"
  done
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --emulate-world 8 --no-cpu-baseline --no-configs --no-variants > $o/emu8.json 2> $o/emu8.err || { echo "emu8 failed"; tail -5 $o/emu8.err; exit 1; }
show $o/emu8.json "emu8 default"

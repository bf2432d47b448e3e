#!/bin/bash
# round 5: A/B of the tail kernels' issue priority (AFM_TAIL_PRIO 0 / 2 / 3) on the headline step
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5m; mkdir -p $o
B=alpha-multi-factor-models_amd/build/exp
for rep in 1 2; do
  for v in default prio3 prio2; do
    if [ $v = default ]; then lib=""; else lib=$R/$B/$v/libafm.so; fi
    AFM_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-configs --no-variants > $o/$v.$rep.json 2> $o/$v.$rep.err || { echo "$v failed"; tail -5 $o/$v.$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$o/$v.$rep.json').read().strip().splitlines()[-1])
print('$v', $rep, d['ms_per_step'], {k: round(v,2) for k,v in d.get('stage_ms',{}).items()})"
  done
done

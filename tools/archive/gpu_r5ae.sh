#!/bin/bash
# round 5: FM grid x fork point on the headline
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5ae; mkdir -p $o
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1])
print('$2', d['ms_per_step'], {k: round(v,2) for k,v in d.get('stage_ms',{}).items()})"; }
for rep in 1 2; do
  for cfg in "0 predict" "512 rebalance" "512 analyzer" "512 gram"; do
    set -- $cfg
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --fm-grid $1 --fm-fork $2 --no-cpu-baseline --no-configs --no-variants > $o/g$1_$2.$rep.json 2> $o/g$1_$2.$rep.err || { echo "$cfg failed"; tail -5 $o/g$1_$2.$rep.err; exit 1; }
    show $o/g$1_$2.$rep.json "fm_grid=$1 fork=$2 $rep"
  done
done

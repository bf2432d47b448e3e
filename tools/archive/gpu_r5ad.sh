#!/bin/bash
# round 5: the FM per-date Grams' persistent grid (one / 1.5 / two workgroups per CU) on the headline
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5ad; mkdir -p $o
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1])
print('$2', d['ms_per_step'], {k: round(v,2) for k,v in d.get('stage_ms',{}).items()})"; }
for rep in 1 2; do
  for g in 0 384 512; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --fm-grid $g --no-cpu-baseline --no-configs --no-variants > $o/g$g.$rep.json 2> $o/g$g.$rep.err || { echo "g=$g failed"; tail -5 $o/g$g.$rep.err; exit 1; }
    show $o/g$g.$rep.json "fm_grid=$g $rep"
  done
done

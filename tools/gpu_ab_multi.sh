#!/bin/bash
# Several bench argument sets on the one-GPU headline step, interleaved repeats:
#   tools/gpu_ab_multi.sh <tag> <reps> "<args 0>" "<args 1>" ...
set -o pipefail
TAG=$1; REPS=$2; shift 2
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/$TAG; mkdir -p $o
for r in $(seq 1 $REPS); do i=0; for args in "$@"; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-variants --no-configs $args > $o/v$i.$r.json 2> $o/v$i.$r.err || { tail -5 $o/v$i.$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/v$i.$r.json').read().strip().splitlines()[-1]); print('v$i', '$args', d['ms_per_step'], {k: round(v, 2) for k, v in d['stage_ms'].items()})"
  i=$((i+1))
done; done

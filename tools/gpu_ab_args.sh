#!/bin/bash
# A/B of two bench argument sets on the one-GPU headline step, interleaved repeats:
#   tools/gpu_ab_args.sh <tag> <reps> "<args A>" "<args B>"
set -o pipefail
TAG=$1; REPS=$2; A=$3; B=$4
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/$TAG; mkdir -p $o
for r in $(seq 1 $REPS); do for v in A B; do
  args=$A; [ $v = B ] && args=$B
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-variants --no-configs $args > $o/$v$r.json 2> $o/$v$r.err || { tail -5 $o/$v$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/$v$r.json').read().strip().splitlines()[-1]); print('$v', '$args', d['ms_per_step'], {k: round(v, 2) for k, v in d['stage_ms'].items()})"
done; done

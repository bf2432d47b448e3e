#!/bin/bash
# A/B of one environment setting on a bench command line, interleaved repeats:
#   tools/gpu_ab_env.sh <tag> <reps> "<VAR=value>" [bench args...]
set -o pipefail
TAG=$1; REPS=$2; ENVB=$3; shift 3
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/$TAG; mkdir -p $o
for r in $(seq 1 $REPS); do for v in A B; do
  if [ $v = B ]; then E="env $ENVB"; else E=""; fi
  timeout -k 10 300 $E python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-variants --no-configs "$@" > $o/$v$r.json 2> $o/$v$r.err || { tail -5 $o/$v$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/$v$r.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], {k: round(v, 2) for k, v in d['stage_ms'].items()})"
done; done

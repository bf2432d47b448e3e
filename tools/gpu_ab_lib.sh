#!/bin/bash
# A/B of an experiment library build against the product library on the headline step,
# interleaved repeats:  tools/gpu_ab_lib.sh <tag> <reps> <variant libafm.so> [bench args...]
set -o pipefail
TAG=$1; REPS=$2; LIBB=$3; shift 3
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/$TAG; mkdir -p $o
for r in $(seq 1 $REPS); do for v in prod var; do
  if [ $v = var ]; then export AFM_LIB=$LIBB; else unset AFM_LIB; fi
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-variants --no-configs "$@" > $o/$v$r.json 2> $o/$v$r.err || { tail -5 $o/$v$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/$v$r.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], {k: round(v, 2) for k, v in d['stage_ms'].items()})"
done; done

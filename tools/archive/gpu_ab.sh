#!/bin/bash
# bench A/B over an env variable: tools/gpu_ab.sh <tag> VAR val1 val2 [val3 ...]
TAG=$1; VAR=$2; shift 2
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in "$@" "$@"; do
  env $VAR=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err || { tail -5 gpurun_out/${TAG}_$v.err; exit 1; }
  echo "$VAR=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_$v.json) $(grep -o '"analyzer": [0-9.]*\|"fm": [0-9.]*\|"pnl": [0-9.]*' gpurun_out/${TAG}_$v.json | tr '\n' ' ')"
done

#!/bin/bash
# bench A/B over values of one environment variable (box): tools/gpu_ab_env.sh VAR "v1 v2 ..." [rounds]
VAR=$1; VALS=$2; R=${3:-1}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in $(seq $R); do for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$v.json 2>/dev/null || exit 1
  echo "$VAR=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$v.json)"
done; done

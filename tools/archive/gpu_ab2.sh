#!/bin/bash
# bench A/B over settings given as "VAR=v,VAR2=w ..." (box): tools/gpu_ab2.sh "<set1> <set2> ..." [rounds]
SETS=$1; R=${2:-1}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in $(seq $R); do for st in $SETS; do
  env $(echo $st | tr ',' ' ') timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab2.json 2>gpurun_out/ab2.err || { tail -5 gpurun_out/ab2.err; exit 1; }
  echo "$st $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab2.json)"
done; done

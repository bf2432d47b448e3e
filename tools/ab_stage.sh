#!/bin/bash
# A/B one stage between two builds of libafm.so on the SAME box, alternating A B A B.
# usage: tools/ab_stage.sh <stage> <libA> <libB> [reps]
st=$1; A=$2; B=$3; n=${4:-2}
for i in $(seq $n); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    printf "%s " $v
    AFM_LIB=$lib timeout -k 10 120 python3 tools/stage_bench.py --stages $st --reps 3 | tail -1 || exit 1
  done
done

#!/bin/bash
# Kernel stats + the last step's timeline (box).  Usage: tools/gpu_tl.sh <tag> [bench args]
TAG=$1; shift
R=$GRAFT_REPO_ROOT; cd $R
tools/gpu_prof.sh $TAG "$@" || exit 1
f=$(find $R/gpurun_out/${TAG}_prof -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_step.py $f > $R/gpurun_out/${TAG}_timeline.txt && head -60 $R/gpurun_out/${TAG}_timeline.txt

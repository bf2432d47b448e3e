#!/bin/bash
# kernel trace of the emulated N-rank step (bench.py --emulate-world N) and its last-step timeline
#   tools/gpu_trace_emu.sh <tag> <N> <factor launches per step> [bench args...]
set -o pipefail
TAG=$1; W=$2; PER=$3; shift 3
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof$W -o run --output-format csv -- \
    python3 $R/bench.py --steps 5 --warmup 2 --emulate-world $W "$@" > $R/gpurun_out/${TAG}_prof$W.log 2>&1 \
    || { echo "prof failed"; tail -20 $R/gpurun_out/${TAG}_prof$W.log; exit 1; }
cd $R
python3 tools/trace_step.py gpurun_out/${TAG}_prof$W/run_kernel_trace.csv $PER > gpurun_out/${TAG}_step_timeline_emu$W.txt
python3 tools/rocprof_summary.py gpurun_out/${TAG}_prof$W/run_kernel_trace.csv > gpurun_out/${TAG}_kernel_stats_emu$W.txt
cat gpurun_out/${TAG}_step_timeline_emu$W.txt

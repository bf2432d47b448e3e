#!/bin/bash
# kernel traces (rocprofv3 --kernel-trace --stats): the headline step and the emulated N=8 rank
#   tools/gpu_prof.sh <tag>
set -o pipefail
TAG=$1; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-variants --no-configs > $R/gpurun_out/${TAG}_prof.log 2>&1 \
    || { echo "prof failed"; tail -20 $R/gpurun_out/${TAG}_prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof8 -o run --output-format csv -- \
    python3 $R/bench.py --steps 5 --warmup 2 --emulate-world 8 > $R/gpurun_out/${TAG}_prof8.log 2>&1 \
    || { echo "prof8 failed"; tail -20 $R/gpurun_out/${TAG}_prof8.log; exit 1; }
cd $R
python3 tools/rocprof_summary.py gpurun_out/${TAG}_prof/run_kernel_trace.csv > gpurun_out/${TAG}_kernel_stats.txt
python3 tools/trace_step.py gpurun_out/${TAG}_prof/run_kernel_trace.csv > gpurun_out/${TAG}_step_timeline.txt
python3 tools/rocprof_summary.py gpurun_out/${TAG}_prof8/run_kernel_trace.csv > gpurun_out/${TAG}_kernel_stats_emu8.txt
head -24 gpurun_out/${TAG}_kernel_stats.txt
head -20 gpurun_out/${TAG}_kernel_stats_emu8.txt

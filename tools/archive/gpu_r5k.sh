#!/bin/bash
# kernel traces (rocprofv3 --kernel-trace --stats) of the config B / D / E bench lines
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in e b d; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5k_$c -o run --output-format csv -- \
      python3 $R/bench.py --config-only $c > $R/gpurun_out/r5k_$c.log 2>&1 || { echo "prof $c failed"; tail -20 $R/gpurun_out/r5k_$c.log; exit 1; }
done
cd $R
for c in e b d; do
  python3 tools/rocprof_summary.py gpurun_out/r5k_$c/run_kernel_trace.csv > gpurun_out/r5k_${c}_kernel_stats.txt
  tail -1 gpurun_out/r5k_$c.log | cut -c1-400
  head -16 gpurun_out/r5k_${c}_kernel_stats.txt
done

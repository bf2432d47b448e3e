#!/bin/bash
# round 5: kernel trace of the emulated world-8 rank step and of the headline (the PnL stage)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
B=$R/alpha-multi-factor-models_amd/build/exp
AFM_LIB=$B/fmmfma/libafm.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5o_emu8 -o run --output-format csv -- \
    python3 $R/bench.py --steps 5 --warmup 2 --emulate-world 8 --no-cpu-baseline --no-configs --no-variants > $R/gpurun_out/r5o_emu8.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/r5o_emu8.log; exit 1; }
AFM_LIB=$B/fmmfma/libafm.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5o_c -o run --output-format csv -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-configs --no-variants > $R/gpurun_out/r5o_c.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/r5o_c.log; exit 1; }
cd $R
for n in emu8 c; do python3 tools/rocprof_summary.py gpurun_out/r5o_$n/run_kernel_trace.csv > gpurun_out/r5o_${n}_kernel_stats.txt; done
head -30 gpurun_out/r5o_emu8_kernel_stats.txt

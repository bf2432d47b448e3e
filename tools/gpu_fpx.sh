#!/bin/bash
# factor-kernel experiments (box): listing spread / fast-step on-off / shard sizes, then PMC
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
o=gpurun_out/fpx; mkdir -p $o
run() { timeout -k 10 200 python -u tools/fp_probe.py "$@" >> $o/probe.log 2>&1 || { tail -5 $o/probe.log; exit 1; }; }
run --listing-frac 0.1 && run --listing-frac 0.0 && run --listing-frac 0.1 --fast 0 && \
run --assets 1250 && run --assets 2500 && run --assets 5000
grep -v amdgpu.ids $o/probe.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES --output-format csv -d $R/$o/pmc_a -o run -- python3 $R/tools/fp_probe.py --reps 1 > $R/$o/pmc_a.log 2>&1 && \
python3 $R/tools/pmc_summary.py $R/$o/pmc_a | grep -E "factor_panel|labels"

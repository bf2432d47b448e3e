set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/fp_pmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/fp_pmc/avail.txt 2>&1
grep -o "SQC_[A-Z_0-9]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT[A-Z_]*\|SQ_INST_LEVEL[A-Z_]*" $R/gpurun_out/fp_pmc/avail.txt | sort -u | head -60
run() { local n=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/fp_pmc/$n -o run -- python3 $R/tools/stage_bench.py --stages factors --reps 1 > $R/gpurun_out/fp_pmc/$n.log 2>&1; }
run a SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES && \
run b SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR
ls $R/gpurun_out/fp_pmc
python3 $R/tools/pmc_summary.py $R/gpurun_out/fp_pmc | grep factor_panel

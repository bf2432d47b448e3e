#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over tools/stage_bench.py for some stages.
# Usage (GPU box, repo root): tools/pmc_stage.sh <outdir> <stages>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/$1; ST=$2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
    python3 $R/tools/stage_bench.py --stages $ST --reps 1 > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $OUT/$name.log; exit 1; }
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run sq2 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES
run fetch FETCH_SIZE
run write WRITE_SIZE
python3 $R/tools/pmc_summary.py $OUT/sq1 $OUT/sq2 $OUT/fetch $OUT/write

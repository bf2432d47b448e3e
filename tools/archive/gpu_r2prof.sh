#!/bin/bash
# Round-2 evidence: kernel stats at top_n 10 and 100, PMC passes (sq1/sq2/fetch/write) at top_n 10.
# Usage (box): tools/gpu_r2prof.sh <tag>
TAG=$1
R=$GRAFT_REPO_ROOT; cd $R
tools/gpu_prof.sh ${TAG}_t10 || exit 1
tools/gpu_prof.sh ${TAG}_t100 --top-n 100 || exit 1
cd $R && tools/prof_counters.sh gpurun_out/${TAG}_pmc || { echo "pmc failed"; exit 1; }
cd $R && python3 tools/pmc_traffic.py gpurun_out/${TAG}_pmc gpurun_out/${TAG}_pmc_traffic.json && \
  python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc/sq1 gpurun_out/${TAG}_pmc/sq2 gpurun_out/${TAG}_pmc/fetch gpurun_out/${TAG}_pmc/write > gpurun_out/${TAG}_pmc.txt && \
  head -c 2500 gpurun_out/${TAG}_pmc.txt

#!/bin/bash
# round-end PMC passes (FETCH_SIZE / WRITE_SIZE and SQ counters) over one headline step
#   tools/gpu_pmc.sh <tag>   -> gpurun_out/<tag>_pmc, <tag>_pmc_traffic.json, <tag>_pmc.txt
set -o pipefail
TAG=${1:-r5w}
R=$GRAFT_REPO_ROOT; cd $R
BENCH_ARGS="--no-variants --no-configs" bash tools/prof_counters.sh gpurun_out/${TAG}_pmc || exit 1
python3 tools/pmc_traffic.py gpurun_out/${TAG}_pmc gpurun_out/${TAG}_pmc_traffic.json 10000 5040 || exit 1
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc > gpurun_out/${TAG}_pmc.txt 2>&1 || exit 1
head -30 gpurun_out/${TAG}_pmc.txt
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_pmc_traffic.json')); [print(k, v) for k, v in d['kernels'].items() if 'factor' in k or 'zgram' in k or 'zscore' in k]"

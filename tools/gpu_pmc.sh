#!/bin/bash
# round-end PMC passes (FETCH_SIZE / WRITE_SIZE and SQ counters) over one headline step
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
BENCH_ARGS="--no-variants" bash tools/prof_counters.sh gpurun_out/r4z_pmc || exit 1
python3 tools/pmc_traffic.py gpurun_out/r4z_pmc gpurun_out/r4z_pmc_traffic.json 10000 5040 || exit 1
python3 tools/pmc_summary.py gpurun_out/r4z_pmc > gpurun_out/r4z_pmc.txt 2>&1 || exit 1
head -30 gpurun_out/r4z_pmc.txt
python3 -c "import json; d=json.load(open('gpurun_out/r4z_pmc_traffic.json')); [print(k, v) for k, v in d['kernels'].items() if 'factor' in k or 'zgram' in k]"

#!/bin/bash
# PMC traffic of the config-D pass (bench.py --config-only d: one warm-up pass + 2 timed passes =
# 3 passes of the time-slab factor build), one rocprofv3 pass per counter group
#   tools/gpu_pmc_config_d.sh <tag>  -> gpurun_out/<tag>_pmc_d/, gpurun_out/<tag>_pmc_config_d.json
set -o pipefail
TAG=${1:-r6}
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/${TAG}_pmc_d; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  n=$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
  timeout -s KILL 400 rocprofv3 --pmc $c --output-format csv -d $OUT/$n -o run -- \
    python3 $R/bench.py --config-only d > $OUT/$n.log 2>&1 || { echo "pmc $c failed"; tail -5 $OUT/$n.log; exit 1; }
done
cd $R
python3 tools/pmc_pass.py gpurun_out/${TAG}_pmc_d gpurun_out/${TAG}_pmc_config_d.json 3 3000 196560 \
    factor_panel_kernel masks_kernel labels_kernel || exit 1

#!/bin/bash
# zscore tests + bench A/B of the stats kernel (2 vs 1 columns per thread).  Usage: tools/gpu_zs.sh <tag>
TAG=$1
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_zscore_gpu.py tests/test_chain_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -2 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/${TAG}_tests.log | head; exit $rc; fi
for v in 2; do
  AFM_ZS_CPT=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_b$v.json 2> gpurun_out/${TAG}_b$v.err || { tail -5 gpurun_out/${TAG}_b$v.err; exit 1; }
  echo "cpt $v"; grep -o '"ms_per_step": [0-9.]*\|"zstats": [0-9.]*' gpurun_out/${TAG}_b$v.json
done

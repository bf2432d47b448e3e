#!/bin/bash
# Analyzer + chain tests and a bench line.  Usage (box): tools/gpu_an.sh <tag>
TAG=$1
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_analyzer_gpu.py tests/test_chain_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -4 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/${TAG}_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/${TAG}_bench.json

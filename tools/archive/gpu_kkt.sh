#!/bin/bash
# Portfolio / KKT tests, the chain tests and a top_n=100 stress bench.  Usage (box): tools/gpu_kkt.sh <tag>
TAG=$1
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_portfolio_gpu.py tests/test_chain_gpu.py tests/test_sharded.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/${TAG}_tests.log | sed 's/ PASSED.*//' | tr '\n' ' ' | head -c 3000; echo
tail -25 gpurun_out/${TAG}_tests.log | grep -v "^$"
if [ $rc -ne 0 ]; then echo "tests ended with $rc"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --top-n 100 > gpurun_out/${TAG}_bench100.json 2> gpurun_out/${TAG}_bench100.err || { tail -20 gpurun_out/${TAG}_bench100.err; exit 1; }
grep warmup gpurun_out/${TAG}_bench100.err
grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/${TAG}_bench100.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
grep warmup gpurun_out/${TAG}_bench.err
grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/${TAG}_bench.json

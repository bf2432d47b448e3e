#!/bin/bash
# Gram probe (numerics + timing), chain / sharded / config tests, bench.  Usage (box): tools/gpu_zb.sh <tag>
TAG=$1
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 240 python -u tools/zgram_probe.py --chunks 64 > gpurun_out/${TAG}_probe.log 2>&1 || { echo "probe failed $?"; tail -5 gpurun_out/${TAG}_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_probe.log
timeout -k 10 600 python -u -m pytest tests/test_chain_gpu.py tests/test_sharded.py tests/test_configs_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/${TAG}_tests.log | head; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/${TAG}_bench.json

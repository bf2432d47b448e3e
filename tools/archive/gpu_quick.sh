#!/bin/bash
# Quick GPU iteration: one test file, then the bench line with the fast path on and off.
# Usage (box, repo root): tools/gpu_quick.sh <tag> [test file]
set -o pipefail
TAG=$1; TF=${2:-tests/test_factors_gpu.py}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest $TF -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
AFM_FP_NOFAST=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_bench_nofast.json 2>&1 \
    || { echo "nofast bench failed"; exit 1; }
grep -o '"stage_ms": {[^}]*}' gpurun_out/${TAG}_bench_nofast.json

#!/bin/bash
# GPU-box check: parity tests, one bench line, a kernel-trace profile of the same bench command.
# Usage (from the repo root on the box): tools/gpu_check.sh <tag> [pytest -k expr]
set -o pipefail
TAG=$1; K=${2:-}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread "${KARG[@]}" \
    > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $R/gpurun_out/${TAG}_prof.log 2>&1 \
    || { echo "prof failed"; tail -20 $R/gpurun_out/${TAG}_prof.log; exit 1; }
python3 $R/tools/rocprof_summary.py $R/gpurun_out/${TAG}_prof/run_kernel_trace.csv | head -16

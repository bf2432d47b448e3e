#!/bin/bash
# round-end style check: every GPU test, smoke, one bench line (with the CPU baseline), a kernel
# trace of the headline step alone (no variant lines) and its step timeline
set -o pipefail
TAG=$1; R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 \
    || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print(d['ms_per_step'], d['value'], d['stage_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-variants > $R/gpurun_out/${TAG}_prof.log 2>&1 \
    || { echo "prof failed"; tail -20 $R/gpurun_out/${TAG}_prof.log; exit 1; }
cd $R
python3 tools/rocprof_summary.py gpurun_out/${TAG}_prof/run_kernel_trace.csv > gpurun_out/${TAG}_kernel_stats.txt
python3 tools/trace_step.py gpurun_out/${TAG}_prof/run_kernel_trace.csv > gpurun_out/${TAG}_step_timeline.txt
head -14 gpurun_out/${TAG}_kernel_stats.txt

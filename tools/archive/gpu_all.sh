#!/bin/bash
# Full GPU test suite + smoke + bench line.  Usage (box): tools/gpu_all.sh <tag>
TAG=$1
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/${TAG}_tests.log | sed 's/ PASSED.*//' | tr '\n' ' ' | head -c 3000; echo
tail -25 gpurun_out/${TAG}_tests.log | grep -v "^$"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc"; exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python -u bench.py --steps ${STEPS:-5} --warmup 2 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
grep warmup gpurun_out/${TAG}_bench.err
grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/${TAG}_bench.json
exit $rc

#!/bin/bash
# GPU box: chain parity tests, then the bench line (stops after any crash / timeout).
# Usage (repo root on the box): tools/gpu_chain.sh <tag> [test files...]
TAG=$1; shift
TESTS=${@:-tests/test_chain_gpu.py}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -25 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps ${STEPS:-3} --warmup ${WARMUP:-1} ${BENCH_ARGS:---no-cpu-baseline} \
    > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc2=$?
tail -5 gpurun_out/${TAG}_bench.err
cat gpurun_out/${TAG}_bench.json
exit $(( rc2 != 0 ? rc2 : rc ))

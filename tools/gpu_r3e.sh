#!/bin/bash
# zstats with the Markstein reciprocal division: parity + step timing
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
o=gpurun_out/r3e; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_zscore_gpu.py tests/test_chain_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-variants > $o/bench.json 2> $o/bench.err || { tail -5 $o/bench.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' $o/bench.json

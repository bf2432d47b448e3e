#!/bin/bash
# zstats Markstein + early FM: parity and step timing (A/B fm_early)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
o=gpurun_out/r3f; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_zscore_gpu.py tests/test_chain_gpu.py tests/test_configs_gpu.py tests/test_sharded.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/stage_ab.py > $o/ab.log 2>&1 || { tail -5 $o/ab.log; exit 1; }
grep -v amdgpu.ids $o/ab.log

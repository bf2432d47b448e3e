#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
tools/gpu_chain.sh $1 tests/test_chain_gpu.py tests/test_analyzer_gpu.py || exit $?
timeout -k 10 200 python -u tools/zgram_probe.py > gpurun_out/$1_probe.log 2>&1 || { tail -20 gpurun_out/$1_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/$1_probe.log

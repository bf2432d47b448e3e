#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_chain_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/c2_tests.log 2>&1
rc=$?; tail -15 gpurun_out/c2_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc"; exit $rc; fi
timeout -k 10 200 python -u tools/zgram_probe.py > gpurun_out/c2_probe.log 2>&1 || { tail -20 gpurun_out/c2_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c2_probe.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c2_bench.json 2> gpurun_out/c2_bench.err || { tail -20 gpurun_out/c2_bench.err; exit 1; }
grep warmup gpurun_out/c2_bench.err; cat gpurun_out/c2_bench.json

#!/bin/bash
# zgram probe: default build (timing + numerics check), then the two skip variants, then a bench line
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python -u tools/zgram_probe.py "$@" > gpurun_out/zg_default.log 2>&1 || { cat gpurun_out/zg_default.log; exit 1; }
grep -v amdgpu.ids gpurun_out/zg_default.log
for v in 1 2; do
  AFM_LIB=$GRAFT_REPO_ROOT/alpha-multi-factor-models_amd/build/zg_skip$v/libafm.so timeout -k 10 200 python -u tools/zgram_probe.py --check 0 "$@" > gpurun_out/zg_skip$v.log 2>&1 || { cat gpurun_out/zg_skip$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/zg_skip$v.log
done
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/zg_bench.json 2> gpurun_out/zg_bench.err || { tail -20 gpurun_out/zg_bench.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/zg_bench.json

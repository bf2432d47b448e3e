#!/bin/bash
# zgram probe: default build (timing + numerics check), then the two skip variants
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python -u tools/zgram_probe.py "$@" > gpurun_out/zg_default.log 2>&1 || { cat gpurun_out/zg_default.log; exit 1; }
cat gpurun_out/zg_default.log | grep -v amdgpu.ids
for v in 1 2; do
  AFM_LIB=$GRAFT_REPO_ROOT/alpha-multi-factor-models_amd/build/zg_skip$v/libafm.so timeout -k 10 200 python -u tools/zgram_probe.py --check 0 "$@" > gpurun_out/zg_skip$v.log 2>&1 || { cat gpurun_out/zg_skip$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/zg_skip$v.log
done

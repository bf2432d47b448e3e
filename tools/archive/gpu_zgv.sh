#!/bin/bash
# zpool code-shape A/B: default build, then every build/zgv/<name>/libafm.so
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python -u tools/zgram_probe.py --check 0 > gpurun_out/zgv_default.log 2>&1 || { cat gpurun_out/zgv_default.log; exit 1; }
echo "default: $(grep zpool gpurun_out/zgv_default.log)"
for d in alpha-multi-factor-models_amd/build/zgv/*/; do
  n=$(basename $d)
  AFM_LIB=$GRAFT_REPO_ROOT/$d/libafm.so timeout -k 10 200 python -u tools/zgram_probe.py --check 0 > gpurun_out/zgv_$n.log 2>&1 || { cat gpurun_out/zgv_$n.log; exit 1; }
  echo "$n: $(grep zpool gpurun_out/zgv_$n.log | sed 's/lib [^:]*: //')"
done

#!/bin/bash
# Factor-kernel A/B (box): the f64 latency probe, then for the default build and each
# build/zgv/<name> in FP_VARIANTS: factor stage times at config C and the bit-exact factor tests.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
if [ -n "$LAT" ] && [ -x tools/lat_probe/lat_probe ]; then
  timeout -k 10 60 tools/lat_probe/lat_probe > gpurun_out/lat_probe.txt 2>&1 || { cat gpurun_out/lat_probe.txt; exit 1; }
  cat gpurun_out/lat_probe.txt
fi
for v in default ${FP_VARIANTS}; do
  if [ $v = default ]; then L=""; else L=$GRAFT_REPO_ROOT/alpha-multi-factor-models_amd/build/zgv/$v/libafm.so; fi
  AFM_LIB=$L timeout -k 10 240 python -u tools/fp_probe.py --reps ${FP_REPS:-5} > gpurun_out/fpab_$v.log 2>&1 || { tail -20 gpurun_out/fpab_$v.log; exit 1; }
  grep factors gpurun_out/fpab_$v.log
  if [ -n "$FP_TEST" ]; then
    AFM_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_factors_gpu.py > gpurun_out/fpab_test_$v.log 2>&1 || { tail -20 gpurun_out/fpab_test_$v.log; exit 1; }
    echo "$v tests: $(tail -1 gpurun_out/fpab_test_$v.log)"
  fi
done

#!/bin/bash
# zpool A/B between library builds under build/zgv/<name> and the default (box)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in default ${ZG_VARIANTS}; do
  if [ $v = default ]; then L=""; else L=$GRAFT_REPO_ROOT/alpha-multi-factor-models_amd/build/zgv/$v/libafm.so; fi
  AFM_LIB=$L timeout -k 10 240 python -u tools/zgram_probe.py --check 0 --chunks 64 > gpurun_out/zgab_$v.log 2>&1 || { tail -20 gpurun_out/zgab_$v.log; exit 1; }
  echo "$v: $(grep -E 'zpool with|fm \(' gpurun_out/zgab_$v.log | tr '\n' ' ' | sed 's/lib [^:]*: //')"
done

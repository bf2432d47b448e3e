#!/bin/bash
# partition p2: parity (factor + intraday tests), per-wave profiles at the N=8 shard size
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4j; mkdir -p $o
P=$R/alpha-multi-factor-models_amd/build/exp
AFM_LIB=$P/p2/libafm.so timeout -k 10 300 python -u -m pytest tests/test_factors_gpu.py tests/test_intraday_gpu.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit 1
for v in p1prof p2prof; do
  AFM_FP_TYPES=15 AFM_LIB=$P/$v/libafm.so timeout -k 10 200 python -u tools/wave_profile.py 1250 > $o/wave1250_$v.txt 2>&1 || { tail -5 $o/wave1250_$v.txt; exit 1; }
  cat $o/wave1250_$v.txt
done
AFM_LIB=$P/p2prof/libafm.so timeout -k 10 200 python -u tools/wave_profile.py > $o/wave_p2prof.txt 2>&1 || { tail -5 $o/wave_p2prof.txt; exit 1; }
cat $o/wave_p2prof.txt

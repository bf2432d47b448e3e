#!/bin/bash
# factor kernel: loader with two chunks of loads in flight; PnL alone
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4f; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_factors_gpu.py tests/test_intraday_gpu.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || exit 1
for A in 10000 1250; do
  timeout -k 10 200 python -u tools/fp_probe.py --assets $A --reps 7 >> $o/fp.txt 2>&1 || exit 1
done
grep -E "factors" $o/fp.txt
AFM_LIB=$R/alpha-multi-factor-models_amd/build/prof/libafm.so timeout -k 10 200 python3 tools/wave_profile.py 10000 5040 > $o/wave_profile.txt 2>&1 || { tail -5 $o/wave_profile.txt; exit 1; }
grep -v amdgpu.ids $o/wave_profile.txt
timeout -k 10 300 python -u tools/pnl_probe.py > $o/pnl.txt 2>&1 || { tail -5 $o/pnl.txt; exit 1; }
grep afm_pnl $o/pnl.txt
timeout -k 10 300 python -u tools/pnl_probe.py --assets 1280 >> $o/pnl.txt 2>&1 || { tail -5 $o/pnl.txt; exit 1; }
grep afm_pnl $o/pnl.txt

#!/bin/bash
# factor kernel with item-level counters instead of workgroup barriers: parity, timing, profile;
# rebalance phases at top_n = 100
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
o=gpurun_out/r3d; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_factors_gpu.py tests/test_intraday_gpu.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 200 python -u tools/fp_probe.py > $o/probe.log 2>&1 && timeout -k 10 200 python -u tools/fp_probe.py --assets 1250 >> $o/probe.log 2>&1 || { tail -5 $o/probe.log; exit 1; }
grep -v amdgpu.ids $o/probe.log
AFM_LIB=$GRAFT_REPO_ROOT/alpha-multi-factor-models_amd/build/prof/libafm.so timeout -k 10 200 python -u tools/wave_profile.py > $o/wave.txt 2>&1 || { tail -5 $o/wave.txt; exit 1; }
cat $o/wave.txt
PROBES=0,1,2,4 AFM_LIB=$GRAFT_REPO_ROOT/alpha-multi-factor-models_amd/build/prof/libafm.so timeout -k 10 200 python -u tools/reb_probe.py > $o/reb.txt 2>&1 || { tail -5 $o/reb.txt; exit 1; }
grep -v amdgpu.ids $o/reb.txt

#!/bin/bash
# round 5: small-grid factor waves with the next day's ring reads issued ahead (AFM_FP_AHEAD) --
# parity (factor / intraday tests) and fp_probe timing against the variant without it
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5ai; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_factors_gpu.py tests/test_intraday_gpu.py > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
V=$R/alpha-multi-factor-models_amd/build/exp/noahead/libafm.so
for A in 1250 2500 3000 5000; do
  for lib in ahead noahead; do
    if [ $lib = noahead ]; then export AFM_LIB=$V; else unset AFM_LIB; fi
    echo "lib=$lib assets=$A" >> $o/fp.txt
    timeout -k 10 120 python -u tools/fp_probe.py --assets $A --reps 5 >> $o/fp.txt 2>&1 || { tail -5 $o/fp.txt; exit 1; }
  done
done
grep -v amdgpu.ids $o/fp.txt

#!/bin/bash
# portfolio GPU tests (MFMA covariance for books > 32), the top_n = 100 step, the factor wave profile
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
o=gpurun_out/r3b; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_portfolio_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -5 $o/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --top-n 100 --no-cpu-baseline --no-variants > $o/t100.json 2> $o/t100.err || { tail -5 $o/t100.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' $o/t100.json
AFM_LIB=$GRAFT_REPO_ROOT/alpha-multi-factor-models_amd/build/prof/libafm.so timeout -k 10 200 python -u tools/wave_profile.py > $o/wave.txt 2>&1 || { tail -5 $o/wave.txt; exit 1; }
cat $o/wave.txt
exit $rc

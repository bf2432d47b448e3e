#!/bin/bash
# factor A/B (15 vs 21 sets, buffer stores) at 10k and the shard sizes; factor GPU tests;
# the one-GPU step at the per-rank asset counts of N = 8 / 4 / 2
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r3n; o=gpurun_out/r3n
for A in 10000 1250; do for round in 1 2; do
  for lib in default alpha-multi-factor-models_amd/build/exp/fp21/libafm.so; do
    if [ "$lib" = default ]; then L=""; else L=$R/$lib; fi
    AFM_LIB=$L timeout -k 10 120 python -u tools/fp_probe.py --assets $A --reps 7 2>&1 | grep "factors" | sed "s|$R/||" || exit 1
  done; done; done
timeout -k 10 300 python -u -m pytest tests/test_factors_gpu.py tests/test_intraday_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for A in 1250 2500 5000; do
  timeout -k 10 150 python -u bench.py --assets $A --steps 10 --warmup 2 --no-cpu-baseline --no-variants 2>/dev/null > $o/b$A.json || exit 1
  python3 -c "import json; d=json.load(open('$o/b$A.json')); print('A=$A', d['ms_per_step'], d['stage_ms'])"
done

#!/bin/bash
# round 4: barrier-free factor kernel (4-day chunks, LDS counters) + batched PnL staging
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4e; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_factors_gpu.py tests/test_intraday_gpu.py tests/test_portfolio_gpu.py tests/test_chain_gpu.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || exit 1
for A in 10000 1250; do
  timeout -k 10 200 python -u tools/fp_probe.py --assets $A --reps 7 >> $o/fp.txt 2>&1 || exit 1
done
grep -E "factors" $o/fp.txt
AFM_LIB=$R/alpha-multi-factor-models_amd/build/prof/libafm.so timeout -k 10 200 python3 tools/wave_profile.py 10000 5040 > $o/wave_profile.txt 2>&1 || { tail -5 $o/wave_profile.txt; exit 1; }
cat $o/wave_profile.txt
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-variants > $o/bench.json 2> $o/bench.err || { tail -5 $o/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/bench.json')); print(d['ms_per_step'], d['stage_ms'], d['roofline']['frac'], d['roofline_next']['frac'])"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --emulate-world 8 > $o/emu8.json 2> $o/emu8.err || { tail -5 $o/emu8.err; exit 1; }
cat $o/emu8.json
for f in rebalance gram; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-variants --fm-fork $f > $o/bench_fork_$f.json 2> $o/bench_fork_$f.err || { tail -5 $o/bench_fork_$f.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/bench_fork_$f.json')); print('fm_fork $f', d['ms_per_step'], d['stage_ms'])"
done

#!/bin/bash
# round 4: paired 16-B factor stores -- factor parity tests, then the kernel alone
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4b; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_factors_gpu.py tests/test_intraday_gpu.py tests/test_portfolio_gpu.py tests/test_chain_gpu.py tests/test_analyzer_gpu.py tests/test_lasso.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -5 $o/tests.log; [ $rc -eq 0 ] || exit 1
for A in 10000 1250; do
  timeout -k 10 200 python -u tools/fp_probe.py --assets $A --reps 7 >> $o/fp.txt 2>&1 || exit 1
done
grep -E "factors|labels" $o/fp.txt
for f in 0 16 32 64; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-variants --fm-free-cus $f > $o/bench_fm$f.json 2> $o/bench_fm$f.err || { tail -5 $o/bench_fm$f.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$o/bench_fm$f.json')); print('fm_free_cus $f', d['ms_per_step'], d['stage_ms'])"
done
for W in 8 4 2; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --emulate-world $W > $o/emu$W.json 2> $o/emu$W.err || { tail -5 $o/emu$W.err; exit 1; }
  cat $o/emu$W.json
done

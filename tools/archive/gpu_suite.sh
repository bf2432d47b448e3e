#!/bin/bash
# full GPU suite + bench line + per-rank proxy + PnL alone (round-4 run r4h)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/suite; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $o/tests.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/pnl_probe.py > $o/pnl.txt 2>&1 || { tail -5 $o/pnl.txt; exit 1; }
grep afm_pnl $o/pnl.txt
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $o/bench.json 2> $o/bench.err || { tail -5 $o/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/bench.json')); print(d['ms_per_step'], d['stage_ms'], d['roofline']['frac'], d['roofline_next']['frac']); print('top100', d['top_n_100']['ms_per_step'], d['top_n_100']['stage_ms']); print('dense', d['dense_lasso']['ms_per_step'], d['dense_lasso']['stage_ms'])"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --emulate-world 8 > $o/emu8.json 2> $o/emu8.err || { tail -5 $o/emu8.err; exit 1; }
cat $o/emu8.json

#!/bin/bash
# round 5: full GPU suite on the PartS tree, factor launch-shape sweep at 3,000 / 5,000 assets,
# the bench line (configs B / D / E) and per-rank proxies
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5e; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -30; exit 1; }
for A in 3000 5000; do
  for sp in 0 103 105 5 3; do
    timeout -k 10 120 python -u tools/fp_probe.py --assets $A --reps 5 --split $sp >> $o/fp.txt 2>&1 || { tail -5 $o/fp.txt; exit 1; }
  done
done
grep factors $o/fp.txt
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $o/bench.json 2> $o/bench.err || { tail -5 $o/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$o/bench.json'))
print(d['ms_per_step'], d['value'], d['stage_ms'])
for k in ('config_b','config_d','config_e'): print(k, d[k].get('ms_per_step', d[k].get('ms_per_pass')), d[k]['value'], d[k].get('stage_ms', ''), d[k]['roofline']['frac'])"
for w in 8 4 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --emulate-world $w > $o/emu$w.json 2> $o/emu$w.err || { tail -5 $o/emu$w.err; exit 1; }
  cat $o/emu$w.json
done

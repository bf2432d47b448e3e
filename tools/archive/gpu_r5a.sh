#!/bin/bash
# round 5, first box: every GPU test (world-8 sharded case added), smoke, the bench line with the
# config B / D / E lines, per-rank proxies
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5a; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -20; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -5 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $o/bench.json 2> $o/bench.err || { tail -5 $o/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$o/bench.json'))
print(d['ms_per_step'], d['value'], d['stage_ms'])
print('roof', d['roofline']['frac'], '| next', d['roofline_next']['frac'])
for k in ('config_b','config_d','config_e'): print(k, json.dumps(d[k])[:600])"
for w in 8 4; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --emulate-world $w > $o/emu$w.json 2> $o/emu$w.err || { tail -5 $o/emu$w.err; exit 1; }
  cat $o/emu$w.json
done

#!/bin/bash
# round-end style run (tools/gpu_roundend.sh <tag>): every GPU test, smoke, the bench line (with CPU baseline and variants), kernel traces
set -o pipefail
TAG=${1:-r4z}
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/$TAG; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -20; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -5 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 600 python -u bench.py > $o/bench.json 2> $o/bench.err || { tail -5 $o/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$o/bench.json')); print(d['ms_per_step'], d['value'], d['stage_ms']); print('roof', d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic'], '| next', d['roofline_next']['kernel'], d['roofline_next']['frac'], d['roofline_next']['traffic']); print('top100', d['top_n_100']['ms_per_step'], d['top_n_100']['stage_ms']); print('dense', d['dense_lasso']['ms_per_step'], d['dense_lasso']['stage_ms']); print('cpu', d['cpu_baseline']['value'])"
bash tools/gpu_prof.sh $TAG || exit 1

#!/bin/bash
# Round-6 GPU runs, one script with steps chosen by name (no per-run copies):
#   tools/gpu_r6.sh <tag> <step> [<step> ...]
# steps: tests (every -m gpu test), smoke, bench (headline line, no variants / configs / CPU
# baseline), full (the round-end bench line), emu (emulated N = 8 / 4 / 2 rank steps), prof
# (kernel traces: tools/gpu_prof.sh), pmc (PMC traffic passes: tools/gpu_pmc.sh), t:<pytest args>
# (one test selection, e.g. t:tests/test_factors_gpu.py).  Each GPU step has its own time limit
# and the script stops at the first failure.
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/$TAG; mkdir -p $o
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $o/tests.log 2>&1
      rc=$?; tail -2 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -30; exit 1; } ;;
    t:*)
      sel=${step#t:}; sel=${sel//,/ }
      timeout -k 10 600 python -u -m pytest $sel -x -q --timeout 300 --timeout-method thread > $o/sel.log 2>&1
      rc=$?; tail -2 $o/sel.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/sel.log | head -30; exit 1; } ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -5 $o/smoke.log; exit 1; }
      tail -1 $o/smoke.log ;;
    bench)
      timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-variants --no-configs > $o/bench.json 2> $o/bench.err || { tail -5 $o/bench.err; exit 1; }
      python3 -c "import json; d=json.load(open('$o/bench.json')); print(d['ms_per_step'], d['value'], 'host', d.get('host_issue_ms_per_step'), {k: round(v, 2) for k, v in d['stage_ms'].items()}); print('roof', d['roofline']['frac'], d['roofline_next']['frac'])" ;;
    full)
      timeout -k 10 900 python -u bench.py > $o/full.json 2> $o/full.err || { tail -5 $o/full.err; exit 1; }
      python3 -c "import json; d=json.load(open('$o/full.json')); print(d['ms_per_step'], d['value'], d['stage_ms']); print('roof', d['roofline']['frac'], d['roofline_next']['frac']); [print(k, json.dumps(d[k])[:300]) for k in ('top_n_100', 'dense_lasso', 'config_b', 'config_d', 'config_e', 'cpu_baseline')]" ;;
    emu)
      for w in 8 4 2; do
        timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --emulate-world $w > $o/emu$w.json 2> $o/emu$w.err || { tail -5 $o/emu$w.err; exit 1; }
        python3 -c "import json; d=json.loads(open('$o/emu$w.json').read().strip().splitlines()[-1]); print('emu$w', d['ms_per_step'], 'host', d.get('host_issue_ms_per_step'), {k: round(v, 2) for k, v in d['stage_ms'].items()})"
      done ;;
    prof) bash tools/gpu_prof.sh $TAG || exit 1 ;;
    pmc) bash tools/gpu_pmc.sh $TAG || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done

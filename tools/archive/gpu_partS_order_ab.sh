set -o pipefail
B=alpha-multi-factor-models_amd/build/exp/fpbase/libafm.so
o=gpurun_out/r6u; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_factors_gpu.py tests/test_intraday_gpu.py -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1; rc=$?; tail -1 $o/tests.log; [ $rc -eq 0 ] || exit 1
for A in 3000 1250; do for r in 1 2; do
  timeout -k 10 200 python -u tools/fp_probe.py --assets $A --reps 5 2>&1 | grep "^lib" | sed 's/^/new /'
  AFM_LIB=$B timeout -k 10 200 python -u tools/fp_probe.py --assets $A --reps 5 2>&1 | grep "^lib" | sed 's/^/old /'
done; done
for r in 1; do
  timeout -k 10 300 python -u bench.py --config-only d > $o/d_new.json 2>/dev/null && python3 -c "import json; d=json.load(open('$o/d_new.json'))['config_d']; print('new D', d['ms_per_pass'], d['roofline']['frac'])"
  AFM_LIB=$B timeout -k 10 300 python -u bench.py --config-only d > $o/d_old.json 2>/dev/null && python3 -c "import json; d=json.load(open('$o/d_old.json'))['config_d']; print('old D', d['ms_per_pass'], d['roofline']['frac'])"
  timeout -k 10 300 python -u bench.py --config-only b > $o/b_new.json 2>/dev/null && python3 -c "import json; d=json.load(open('$o/b_new.json'))['config_b']; print('new B', d['ms_per_step'], d['stage_ms']['factors'])"
  AFM_LIB=$B timeout -k 10 300 python -u bench.py --config-only b > $o/b_old.json 2>/dev/null && python3 -c "import json; d=json.load(open('$o/b_old.json'))['config_b']; print('old B', d['ms_per_step'], d['stage_ms']['factors'])"
done

#!/bin/bash
# round 5: FM per-date Grams with 2 vs 3 consumer waves (AFM_ZG2_NCW) on the headline
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5af; mkdir -p $o
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1])
print('$2', d['ms_per_step'], {k: round(v,2) for k,v in d.get('stage_ms',{}).items()})"; }
V=$R/alpha-multi-factor-models_amd/build/exp/ncw2/libafm.so
AFM_LIB=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_zgram_wide_gpu.py tests/test_regression_gpu.py > $o/tests.log 2>&1 || { echo "tests failed"; tail -20 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for rep in 1 2; do
  for v in ncw3 ncw2; do
    if [ $v = ncw2 ]; then export AFM_LIB=$V; else unset AFM_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-configs --no-variants > $o/$v.$rep.json 2> $o/$v.$rep.err || { echo "$v failed"; tail -5 $o/$v.$rep.err; exit 1; }
    show $o/$v.$rep.json "$v $rep"
  done
done

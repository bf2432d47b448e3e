#!/bin/bash
# Factor kernel A/B: time + checksum of variant libraries (separate processes, alternating),
# then the factor / intraday / chain GPU tests on the in-tree library.
# Usage (box): tools/gpu_fpab.sh <tag> <libA> [<libB> ...]   (libs relative to the repo root;
# "default" = the in-tree library)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
TAG=$1; shift
o=gpurun_out/$TAG; mkdir -p $o
for round in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = default ]; then L=""; else L=$R/$lib; fi
    AFM_LIB=$L timeout -k 10 200 python -u tools/fp_probe.py --reps 5 >> $o/fp.log 2>&1 \
      || { echo "fp_probe failed ($lib)"; tail -20 $o/fp.log; exit 1; }
  done
done
grep -v amdgpu.ids $o/fp.log | grep -v "^labels"
if [ -n "$FPAB_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest $FPAB_TESTS -x -q -m gpu --timeout 200 --timeout-method thread \
      > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
  tail -2 $o/tests.log
fi

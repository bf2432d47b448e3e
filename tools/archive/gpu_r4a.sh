#!/bin/bash
# round 4: factor-kernel store experiments (store probe patterns + kernel store-mode variants)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r4a; mkdir -p $o
P=alpha-multi-factor-models_amd/build/exp
for m in 0 64 128; do
  timeout -k 10 60 tools/store_probe/store_probe 5040 10000 $m | tail -2 >> $o/probe.txt || exit 1
done
timeout -k 10 60 tools/store_probe/store_probe 5040 10000 16 | tail -1 >> $o/probe.txt || exit 1
cat $o/probe.txt
for lib in default $P/sm1/libafm.so $P/sm2/libafm.so $P/sm3/libafm.so; do
  if [ "$lib" = default ]; then L=""; else L=$R/$lib; fi
  for A in 10000 1250; do
    AFM_LIB=$L timeout -k 10 200 python -u tools/fp_probe.py --assets $A --reps 7 >> $o/fp.txt 2>&1 || exit 1
  done
done
grep -E "factors|labels" $o/fp.txt

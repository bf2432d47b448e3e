#!/bin/bash
# Hot-loop instruction census of each job set of the 30-set small-grid partition (PartS): the
# kernel compiled with one set's code only (-DAFM_FP_ONLY=k), tools/isa_loops.py on its J = 3
# instance; prints, per set, the day loops' VALU counts (the smallest with stores = the clean
# fast step) and scratch / vmcnt waits.
R=$(cd $(dirname $0)/.. && pwd); P=$R/alpha-multi-factor-models_amd
D=/tmp/pack_census_s; mkdir -p $D
for k in $(seq 0 29); do
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I$R/include -I$P/csrc \
      --cuda-device-only -S $AFM_CENSUS_FLAGS -DAFM_FP_ONLY=$k -o $D/s$k.s $P/csrc/factors.hip 2>/dev/null
    python3 $R/tools/isa_loops.py $D/s$k.s factor_panel_kernelINS0_5PartSELi10ELb0E 8 > $D/s$k.txt ) &
  if (( (k + 1) % 6 == 0 )); then wait; fi
done
wait
for k in $(seq 0 29); do
  echo "S$k $(grep 'loop' $D/s$k.txt | grep -v 'stores 0 ' | sed 's/.*instr, VALU \([0-9]*\) (f64 \([0-9]*\).*stores \([0-9]*\).*scratch \([0-9]*\), vmcnt waits \([0-9]*\).*/\1\/\2\/s\4\/w\5/' | sort -t/ -k1 -n | tr '\n' ' ')"
done

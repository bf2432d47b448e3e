#!/bin/bash
# Hot-loop instruction census of each factor job set (W0..W14): the kernel compiled with one set's
# code only (-DAFM_FP_ONLY=k, extra defines in $AFM_CENSUS_FLAGS), then tools/isa_loops.py on its
# <3,true> instance; prints each set's largest loop (the day loop).
R=$(cd $(dirname $0)/.. && pwd); P=$R/alpha-multi-factor-models_amd
D=/tmp/pack_census$1; mkdir -p $D
for k in $(seq 0 14); do
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I$R/include -I$P/csrc \
      --cuda-device-only -S $AFM_CENSUS_FLAGS -DAFM_FP_ONLY=$k -o $D/w$k.s $P/csrc/factors.hip 2>/dev/null
    python3 $R/tools/isa_loops.py $D/w$k.s factor_panel_kernelILi3ELb1 40 > $D/w$k.txt ) &
  if (( (k + 1) % 5 == 0 )); then wait; fi
done
wait
for k in $(seq 0 14); do
  echo "W$k $(grep 'loop' $D/w$k.txt | sort -t'[' -k1 | awk '{print $0}' | python3 -c '
import sys,re
best=None
for l in sys.stdin:
    m=re.search(r"\[(\d+)-(\d+)\]: (\d+) instr, VALU (\d+) \(f64 (\d+).*scratch (\d+)",l)
    if m:
        n=int(m.group(2))-int(m.group(1))
        if best is None or n>best[0]: best=(n,m.group(3),m.group(4),m.group(5),m.group(6))
print("instr %s VALU %s f64 %s scratch %s"%best[1:] if best else "?")')"
done

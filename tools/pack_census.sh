#!/bin/bash
# Hot-loop instruction census of each factor job set (W0..W14): the kernel compiled with one set's
# code only (-DAFM_FP_ONLY=k), then tools/isa_loops.py on its <3,true> instance.
R=$(cd $(dirname $0)/.. && pwd); P=$R/alpha-multi-factor-models_amd
mkdir -p /tmp/pack_census
for k in $(seq 0 14); do
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I$R/include -I$P/csrc \
      --cuda-device-only -S -DAFM_FP_ONLY=$k -o /tmp/pack_census/w$k.s $P/csrc/factors.hip 2>/dev/null
    echo "W$k $(python3 $R/tools/isa_loops.py /tmp/pack_census/w$k.s factor_panel_kernelILi3ELb1 40 | grep 'scratch 0, vmcnt waits 0' | grep -v 'stores 0' | head -1)" ) &
  if (( (k + 1) % 5 == 0 )); then wait; fi
done
wait

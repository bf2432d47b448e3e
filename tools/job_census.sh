#!/bin/bash
# Hot-loop VALU of each factor job alone (as job set W0, -DAFM_FP_ONLY=0).
R=$(cd $(dirname $0)/.. && pwd); P=$R/alpha-multi-factor-models_amd
mkdir -p /tmp/job_census
i=0
for j in "Sma<30>" "Ema<30>" "Vwma<30>" "Bbands<32>" "MomAccelRocr<32>" "Macd<24>" "Rsi<14>" "PvtObvPsy" "RetSd3" "RetSd5x15" "VolSd3" "VolSd5x15" "Corr<5, true>" "Corr<15, false>" "Sma<30>, Ema<30>"; do
  ( n=$(echo "$j" | tr -c 'A-Za-z0-9' '_')
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I$R/include -I$P/csrc \
      --cuda-device-only -S -DAFM_FP_ONLY=0 "-DAFM_FP_CENSUS_W0=$j" -o /tmp/job_census/$n.s $P/csrc/factors.hip 2>/dev/null
    echo "$j | $(python3 $R/tools/isa_loops.py /tmp/job_census/$n.s factor_panel_kernelILi3ELb1 5 | grep 'scratch 0, vmcnt waits 0' | grep -v 'stores 0' | sed 's/.*instr, VALU \([0-9]*\) (f64 \([0-9]*\).*stores \([0-9]*\).*/\1 \2 \3/' | sort -n | head -1)" ) &
  i=$((i+1)); if (( i % 5 == 0 )); then wait; fi
done
wait

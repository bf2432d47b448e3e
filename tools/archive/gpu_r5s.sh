#!/bin/bash
# round 5: per-wave cycle profiles of the 60-set partition (codes 212 / 210 / 206) and PartS (110)
# at 1,250 assets, and fp_probe of codes 210 / 206 there
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5s; mkdir -p $o
P=$R/alpha-multi-factor-models_amd/build/prof/libafm.so
for c in 212 210 206 110; do
  AFM_LIB=$P AFM_FP_TYPES=$c timeout -k 10 200 python -u tools/wave_profile.py 1250 5040 > $o/wp_$c.txt 2>&1 || { echo "wp $c failed"; tail -5 $o/wp_$c.txt; exit 1; }
  echo "== $c"; grep -v amdgpu.ids $o/wp_$c.txt
done
for sp in 210 206; do
  timeout -k 10 200 python -u tools/fp_probe.py --assets 1250 --listing-frac 0.1 --reps 5 --split $sp > $o/fp_1250_$sp.txt 2>&1 || exit 1
  tail -1 $o/fp_1250_$sp.txt
done

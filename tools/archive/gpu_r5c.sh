#!/bin/bash
# per-wave cycle profiles of the 30-set partition (profiling build) at 1,250 and 3,000 assets
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5c; mkdir -p $o
L=$R/alpha-multi-factor-models_amd/build/prof/libafm.so
AFM_LIB=$L AFM_FP_TYPES=110 timeout -k 10 120 python -u tools/wave_profile.py 1250 > $o/wp1250.txt 2>&1 || { tail -5 $o/wp1250.txt; exit 1; }
AFM_LIB=$L AFM_FP_TYPES=105 timeout -k 10 120 python -u tools/wave_profile.py 3000 > $o/wp3000.txt 2>&1 || { tail -5 $o/wp3000.txt; exit 1; }
AFM_LIB=$L AFM_FP_TYPES=110 timeout -k 10 120 python -u tools/wave_profile.py 3000 > $o/wp3000_110.txt 2>&1 || { tail -5 $o/wp3000_110.txt; exit 1; }
cat $o/wp1250.txt $o/wp3000.txt $o/wp3000_110.txt

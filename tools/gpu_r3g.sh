#!/bin/bash
# A/B (separate processes): fm_early vs fm_late; factor setprio variant vs product
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
o=gpurun_out/r3g; mkdir -p $o
timeout -k 10 400 python -u tools/stage_ab.py --rounds 2 > $o/ab_fm.log 2>&1 || { tail -5 $o/ab_fm.log; exit 1; }
cat $o/ab_fm.log
timeout -k 10 400 python -u tools/stage_ab.py --rounds 2 --lib-b $GRAFT_REPO_ROOT/alpha-multi-factor-models_amd/build/exp/prio/libafm.so > $o/ab_prio.log 2>&1 || { tail -5 $o/ab_prio.log; exit 1; }
cat $o/ab_prio.log

#!/bin/bash
# Round-2 kernel experiments (box): the chain tests (incl. the pooled-Gram kernel identity), the
# pooled Gram with each kernel (AFM_ZG_DMA), the z-statistics variants (AFM_ZS_G).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_chain_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/exp_chain.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/exp_chain.log | tail -8
[ $rc -ne 0 ] && { tail -30 gpurun_out/exp_chain.log; exit $rc; }
for v in 1 0; do
  AFM_ZG_DMA=$v timeout -k 10 240 python -u tools/zgram_probe.py --check $v --chunks 64 > gpurun_out/exp_zg$v.log 2>&1 || { tail -20 gpurun_out/exp_zg$v.log; exit 1; }
  echo "AFM_ZG_DMA=$v: $(grep -E 'zpool|rel err' gpurun_out/exp_zg$v.log | tr '\n' ' ')"
done
for g in ${ZS_VARIANTS:-0 1 2 4}; do
  AFM_ZS_G=$g timeout -k 10 240 python -u tools/zs_probe.py > gpurun_out/exp_zs$g.log 2>&1 || { tail -20 gpurun_out/exp_zs$g.log; exit 1; }
  grep zstats gpurun_out/exp_zs$g.log
done

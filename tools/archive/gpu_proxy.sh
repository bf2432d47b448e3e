#!/bin/bash
# per-rank proxies (bench.py --emulate-world N, no profiler) for N = 8, 4, 2
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/proxy; mkdir -p $o
for w in 8 4 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --emulate-world $w > $o/emu$w.json 2> $o/emu$w.err || { tail -5 $o/emu$w.err; exit 1; }
  cat $o/emu$w.json
done

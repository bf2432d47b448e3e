#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run; summary per kernel
# Usage (box): tools/gpu_prof.sh <tag> [bench args]
TAG=$1; shift
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $R/gpurun_out/${TAG}_prof.log 2>&1 \
    || { echo "prof failed"; tail -20 $R/gpurun_out/${TAG}_prof.log; exit 1; }
f=$(find $R/gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
print('%-60s %6s %10s %10s'%('kernel','calls','avg_us','total_ms'))
for r in rows[:30]:
    print('%-60s %6s %10.1f %10.2f'%(r['Name'][:60],r['Calls'],float(r['AverageNs'])/1e3,float(r['TotalDurationNs'])/1e6))
" | tee $R/gpurun_out/${TAG}_kernels.txt
grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/${TAG}_prof.log

#!/bin/bash
# kernel split of afm_pnl_scan_f64 (turnover_terms_kernel vs pnl_scan_kernel) on the bench workload
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/r4r
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4r/prof -o run --output-format csv -- \
    python3 $R/tools/pnl_probe.py --reps 20 > $R/gpurun_out/r4r/probe.log 2>&1 || { tail -5 $R/gpurun_out/r4r/probe.log; exit 1; }
cd $R
python3 tools/rocprof_summary.py gpurun_out/r4r/prof/run_kernel_trace.csv > gpurun_out/r4r/stats.txt
grep -E "turnover|pnl_scan|rebalance" gpurun_out/r4r/stats.txt
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r4r/prof/run_kernel_trace.csv')))
for name in ('turnover_terms_kernel','pnl_scan_kernel'):
    d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6 for r in rows if name in r['Kernel_Name']]
    print(name, len(d), ' '.join(f'{x:.3f}' for x in d[-12:]))
PY

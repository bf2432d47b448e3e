#!/bin/bash
# round 5: z statistics streamed behind the factor slabs on the smallest grids -- parity (stream
# placement bit-identity, chain, sharded, configs, intraday, zscore), then the emulated rank steps
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/r5z; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_chain_gpu.py tests/test_sharded.py tests/test_configs_gpu.py tests/test_zscore_gpu.py tests/test_regression_gpu.py tests/test_analyzer_gpu.py -x -v -m gpu --timeout 400 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $o/tests.log | head -30; exit 1; }
show() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1])
print('$2', d['ms_per_step'], {k: round(v,2) for k,v in d.get('stage_ms',{}).items()})"; }
for w in 8 4 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --emulate-world $w --no-cpu-baseline --no-configs --no-variants > $o/emu$w.json 2> $o/emu$w.err || { echo "emu$w failed"; tail -5 $o/emu$w.err; exit 1; }
  show $o/emu$w.json "emu$w"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5z_prof8 -o run --output-format csv -- \
    python3 $R/bench.py --steps 5 --warmup 2 --emulate-world 8 --no-cpu-baseline --no-configs --no-variants > $R/gpurun_out/r5z_prof8.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/r5z_prof8.log; exit 1; }
cd $R; python3 tools/trace_step.py gpurun_out/r5z_prof8/run_kernel_trace.csv > gpurun_out/r5z_step_timeline_emu8.txt; head -40 gpurun_out/r5z_step_timeline_emu8.txt

#!/bin/bash
# Lasso sparse sweeps (parity tests + the dense variant), top_n = 100 kernel stats
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
o=gpurun_out/r3c; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_lasso.py tests/test_chain_gpu.py tests/test_configs_gpu.py::test_config_c_pooled_gram_lasso_predict -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $o/bench.json 2> $o/bench.err || { tail -5 $o/bench.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$o/bench.json').read().strip().splitlines()[-1])
print('headline', d['ms_per_step'], d['stage_ms'])
for k in ('top_n_100','dense_lasso'): print(k, d[k]['ms_per_step'], d[k]['lasso_nnz'], d[k]['lasso_n_iter'], d[k]['stage_ms'])"
bash tools/gpu_prof.sh r3c_t100 --top-n 100 --no-variants > /dev/null 2>&1 || echo "prof failed"
head -16 gpurun_out/r3c_t100_kernels.txt

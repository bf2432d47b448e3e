#!/bin/bash
# Lasso / chain / config GPU tests, then one bench line (headline + variant keys) without the CPU leg
R=$GRAFT_REPO_ROOT; cd $R; o=gpurun_out/${1:-r3o}; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_lasso.py tests/test_chain_gpu.py tests/test_configs_gpu.py -x -q -m gpu \
    --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $o/bench.json 2> $o/bench.err \
    || { tail -20 $o/bench.err; exit 1; }
python3 - $o/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(d["ms_per_step"], d["stage_ms"])
for k in ("dense_lasso", "top_n_100"):
    e = d[k]
    print(k, e["ms_per_step"], e["stage_ms"], e.get("lasso_n_iter"), e.get("lasso_nnz"))
PY

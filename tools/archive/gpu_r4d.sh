#!/bin/bash
# kernel traces + factor-kernel per-wave profile + factor PMC passes
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_prof.sh r4c || exit 1
AFM_LIB=$R/alpha-multi-factor-models_amd/build/prof/libafm.so timeout -k 10 200 python3 tools/wave_profile.py 10000 5040 > gpurun_out/r4c_wave_profile.txt 2>&1 || { tail -5 gpurun_out/r4c_wave_profile.txt; exit 1; }
cat gpurun_out/r4c_wave_profile.txt
bash tools/pmc_factor.sh > gpurun_out/r4c_pmc_factor.txt 2>&1 || { tail -5 gpurun_out/r4c_pmc_factor.txt; exit 1; }
tail -5 gpurun_out/r4c_pmc_factor.txt
for f in 4 8 16; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-variants --fm-free-cus $f > gpurun_out/r4c_bench_fm$f.json 2> gpurun_out/r4c_bench_fm$f.err || { tail -5 gpurun_out/r4c_bench_fm$f.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r4c_bench_fm$f.json')); print('fm_free_cus $f', d['ms_per_step'], d['stage_ms'])"
done
timeout -k 10 300 python -u -m pytest tests/test_chain_gpu.py -q -x --timeout 200 --timeout-method thread -k placement > gpurun_out/r4c_place.log 2>&1; tail -2 gpurun_out/r4c_place.log

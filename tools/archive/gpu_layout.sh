#!/bin/bash
# factor-kernel layout search (box): per-type max Mcycles for each AFM_FP_LAYOUT
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
AFM_FP_LAYOUT=021435021435023415123405021435021435 AFM_LIB=$GRAFT_REPO_ROOT/alpha-multi-factor-models_amd/build/prof/libafm.so timeout -k 10 200 python -u tools/wave_profile.py > gpurun_out/lay_cur.txt 2>&1 || { tail -5 gpurun_out/lay_cur.txt; exit 1; }
echo "cur 021435021435023415123405021435021435: $(grep "max total" gpurun_out/lay_cur.txt)"
AFM_FP_LAYOUT=032145032145203145203145032145032145 AFM_LIB=$GRAFT_REPO_ROOT/alpha-multi-factor-models_amd/build/prof/libafm.so timeout -k 10 200 python -u tools/wave_profile.py > gpurun_out/lay_r1.txt 2>&1 || { tail -5 gpurun_out/lay_r1.txt; exit 1; }
echo "r1 032145032145203145203145032145032145: $(grep "max total" gpurun_out/lay_r1.txt)"
AFM_FP_LAYOUT=031245031245102345102345132045132045 AFM_LIB=$GRAFT_REPO_ROOT/alpha-multi-factor-models_amd/build/prof/libafm.so timeout -k 10 200 python -u tools/wave_profile.py > gpurun_out/lay_r2.txt 2>&1 || { tail -5 gpurun_out/lay_r2.txt; exit 1; }
echo "r2 031245031245102345102345132045132045: $(grep "max total" gpurun_out/lay_r2.txt)"
AFM_FP_LAYOUT=031425031425012345012345031245031245 AFM_LIB=$GRAFT_REPO_ROOT/alpha-multi-factor-models_amd/build/prof/libafm.so timeout -k 10 200 python -u tools/wave_profile.py > gpurun_out/lay_r3.txt 2>&1 || { tail -5 gpurun_out/lay_r3.txt; exit 1; }
echo "r3 031425031425012345012345031245031245: $(grep "max total" gpurun_out/lay_r3.txt)"
AFM_FP_LAYOUT=132045132045103245103245031425031425 AFM_LIB=$GRAFT_REPO_ROOT/alpha-multi-factor-models_amd/build/prof/libafm.so timeout -k 10 200 python -u tools/wave_profile.py > gpurun_out/lay_r4.txt 2>&1 || { tail -5 gpurun_out/lay_r4.txt; exit 1; }
echo "r4 132045132045103245103245031425031425: $(grep "max total" gpurun_out/lay_r4.txt)"

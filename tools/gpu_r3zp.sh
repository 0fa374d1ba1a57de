#!/bin/bash
# k_kpp_int staged-Rig variants at C3 (ROMS_GPU_KPP_TY 0 / 4 / 8 / 43), their
# bitwise test, interleaved twice.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "kpp_int_staged" -x -q --timeout 200 --timeout-method thread > $O/tests_r3zp.log 2>&1 || { tail -30 $O/tests_r3zp.log; exit 1; }
tail -1 $O/tests_r3zp.log
bash tools/ab_env.sh r3zp "--workload c3 --steps 10 --warmup 2" "ROMS_GPU_KPP_TY=0" "ROMS_GPU_KPP_TY=4" "ROMS_GPU_KPP_TY=8" "ROMS_GPU_KPP_TY=43" "ROMS_GPU_KPP_TY=0" "ROMS_GPU_KPP_TY=4" "ROMS_GPU_KPP_TY=8" "ROMS_GPU_KPP_TY=43" > $O/ab_r3zp_c3.txt 2>&1 || { cat $O/ab_r3zp_c3.txt; exit 1; }
cat $O/ab_r3zp_c3.txt

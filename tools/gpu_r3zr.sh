#!/bin/bash
# t3dmix with staged windows (ROMS_GPU_T3DMIX_STG 0 vs 1): bitwise test, then C3 and C2 A/B.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "t3dmix_staged or visc3d_staged" -x -q --timeout 200 --timeout-method thread > $O/tests_r3zr.log 2>&1 || { tail -30 $O/tests_r3zr.log; exit 1; }
tail -1 $O/tests_r3zr.log
bash tools/ab_env.sh r3zr3 "--workload c3 --steps 10 --warmup 2" "ROMS_GPU_T3DMIX_STG=0" "ROMS_GPU_T3DMIX_STG=1" "ROMS_GPU_T3DMIX_STG=0" "ROMS_GPU_T3DMIX_STG=1" > $O/ab_r3zr_c3.txt 2>&1 || { cat $O/ab_r3zr_c3.txt; exit 1; }
cat $O/ab_r3zr_c3.txt
bash tools/ab_env.sh r3zr2 "--steps 30 --warmup 3" "ROMS_GPU_T3DMIX_STG=0" "ROMS_GPU_T3DMIX_STG=1" "ROMS_GPU_T3DMIX_STG=0" "ROMS_GPU_T3DMIX_STG=1" > $O/ab_r3zr_c2.txt 2>&1 || { cat $O/ab_r3zr_c2.txt; exit 1; }
cat $O/ab_r3zr_c2.txt

#!/bin/bash
# visc3d with staged raw windows (ROMS_GPU_VISC_STG 0 vs 1): bitwise test,
# then C3 and C2 A/B interleaved twice.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "visc3d_staged" -x -q --timeout 200 --timeout-method thread > $O/tests_r3zq.log 2>&1 || { tail -30 $O/tests_r3zq.log; exit 1; }
tail -1 $O/tests_r3zq.log
bash tools/ab_env.sh r3zq3 "--workload c3 --steps 10 --warmup 2" "ROMS_GPU_VISC_STG=0" "ROMS_GPU_VISC_STG=1" "ROMS_GPU_VISC_STG=0" "ROMS_GPU_VISC_STG=1" > $O/ab_r3zq_c3.txt 2>&1 || { cat $O/ab_r3zq_c3.txt; exit 1; }
cat $O/ab_r3zq_c3.txt
bash tools/ab_env.sh r3zq2 "--steps 30 --warmup 3" "ROMS_GPU_VISC_STG=0" "ROMS_GPU_VISC_STG=1" "ROMS_GPU_VISC_STG=0" "ROMS_GPU_VISC_STG=1" > $O/ab_r3zq_c2.txt 2>&1 || { cat $O/ab_r3zq_c2.txt; exit 1; }
cat $O/ab_r3zq_c2.txt

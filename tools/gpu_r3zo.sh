#!/bin/bash
# Round-3 late check: full GPU suite + smoke + default bench, then A/Bs at C3
# and C2: k_prsgrd_uv tile rows (ROMS_GPU_PRS_TY 4 vs 8) and the staged-Rig
# k_kpp_int (ROMS_GPU_KPP_TY 0 vs 4, C3 only: C2 has no KPP).
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
bash tools/gpu_suite.sh r3_zo || exit 1
bash tools/ab_env.sh r3zo3 "--workload c3 --steps 10 --warmup 2" "ROMS_GPU_PRS_TY=4" "ROMS_GPU_PRS_TY=8" "ROMS_GPU_KPP_TY=4" "ROMS_GPU_PRS_TY=4" "ROMS_GPU_PRS_TY=8" "ROMS_GPU_KPP_TY=4" > $O/ab_r3zo_c3.txt 2>&1 || { cat $O/ab_r3zo_c3.txt; exit 1; }
cat $O/ab_r3zo_c3.txt
bash tools/ab_env.sh r3zo2 "--steps 30 --warmup 3" "ROMS_GPU_PRS_TY=4" "ROMS_GPU_PRS_TY=8" "ROMS_GPU_PRS_TY=4" "ROMS_GPU_PRS_TY=8" > $O/ab_r3zo_c2.txt 2>&1 || { cat $O/ab_r3zo_c2.txt; exit 1; }
cat $O/ab_r3zo_c2.txt

#!/bin/bash
# Round-3 final refresh: full GPU suite, smoke, default bench line, the
# t3dmix staging A/B (C3, C2), kernel traces (C3, C2) and PMC traffic tables.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
bash tools/gpu_suite.sh r3_zs || exit 1
bash tools/ab_env.sh r3zs3 "--workload c3 --steps 10 --warmup 2" "ROMS_GPU_T3DMIX_STG=0" "ROMS_GPU_T3DMIX_STG=1" "ROMS_GPU_T3DMIX_STG=0" "ROMS_GPU_T3DMIX_STG=1" > $O/ab_r3zs_c3.txt 2>&1 || { cat $O/ab_r3zs_c3.txt; exit 1; }
cat $O/ab_r3zs_c3.txt
bash tools/ab_env.sh r3zs2 "--steps 30 --warmup 3" "ROMS_GPU_T3DMIX_STG=0" "ROMS_GPU_T3DMIX_STG=1" "ROMS_GPU_T3DMIX_STG=0" "ROMS_GPU_T3DMIX_STG=1" > $O/ab_r3zs_c2.txt 2>&1 || { cat $O/ab_r3zs_c2.txt; exit 1; }
cat $O/ab_r3zs_c2.txt
bash tools/gpu_kt.sh r3_zsc3 c3 > /dev/null || { echo KT3FAIL; exit 1; }
bash tools/gpu_kt.sh r3_zsc2 c2 > /dev/null || { echo KT2FAIL; exit 1; }
echo traces done
bash tools/gpu_pmc_traffic.sh > $O/pmc_r3_zs.log 2>&1 || { echo PMCFAIL; tail -10 $O/pmc_r3_zs.log; exit 1; }
echo all done

#!/bin/bash
# Round-3 closing tree: full GPU suite, smoke, default bench line, kernel
# traces (C3, C2) and the PMC traffic tables, with the staged t3dmix default.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
bash tools/gpu_suite.sh r3_zt || exit 1
bash tools/gpu_kt.sh r3_ztc3 c3 > /dev/null || { echo KT3FAIL; exit 1; }
bash tools/gpu_kt.sh r3_ztc2 c2 > /dev/null || { echo KT2FAIL; exit 1; }
echo traces done
bash tools/gpu_pmc_traffic.sh > $O/pmc_r3_zt.log 2>&1 || { echo PMCFAIL; tail -10 $O/pmc_r3_zt.log; exit 1; }
echo all done

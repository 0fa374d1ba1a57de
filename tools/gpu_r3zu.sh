#!/bin/bash
# uv2 edge-column kernels with chunked loads: full suite, smoke, bench, C3/C2 traces, PMC tables.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
bash tools/gpu_suite.sh r3_zu || exit 1
bash tools/gpu_kt.sh r3_zuc3 c3 > /dev/null || { echo KT3FAIL; exit 1; }
bash tools/gpu_kt.sh r3_zuc2 c2 > /dev/null || { echo KT2FAIL; exit 1; }
echo traces done
bash tools/gpu_pmc_traffic.sh > $O/pmc_r3_zu.log 2>&1 || { echo PMCFAIL; tail -10 $O/pmc_r3_zu.log; exit 1; }
echo all done

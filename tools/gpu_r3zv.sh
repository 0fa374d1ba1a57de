#!/bin/bash
# uv2 edge flux third pass chunked: the uv2/basin GPU tests, then C3 bench and trace.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_obc.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/tests_r3zv.log 2>&1 || { tail -30 $O/tests_r3zv.log; exit 1; }
tail -1 $O/tests_r3zv.log
bash tools/gpu_kt.sh r3_zvc3 c3 > /dev/null || { echo KT3FAIL; exit 1; }
grep -E "uv2|busy" $O/kt_r3_zvc3.txt

#!/bin/bash
# One GPU round trip: parity tests, then a profiled short bench.
# usage (on the box): bash tools/gpu_check.sh TAG
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python -m pytest $R/tests -m gpu -x -q > $R/gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
tail -3 $R/gpurun_out/gpu_tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python $R/bench.py --steps 10 --warmup 2 > $R/gpurun_out/prof_$TAG.log 2>&1

#!/bin/bash
# Kernel-trace profile of one bench workload on the box.
# usage: bash tools/gpu_trace.sh TAG [bench args...]
TAG=${1:-x}; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- \
  python $R/bench.py --no-cpu-baseline "$@" > $O/prof_$TAG.json 2> $O/prof_$TAG.err || exit $?
python $R/tools/prof_summary.py $(ls $O/prof_$TAG/*/run_kernel_trace.csv $O/prof_$TAG/run_kernel_trace.csv 2>/dev/null | head -1) \
  --steps 3 --marker "k_step3d_t_h(" > $O/prof_$TAG.txt

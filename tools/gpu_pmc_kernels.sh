#!/bin/bash
# Per-kernel traffic of one bench workload: kernel trace + FETCH + WRITE passes (eager, no graphs).
# usage: bash tools/gpu_pmc_kernels.sh TAG [bench args...]
TAG=${1:-x}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export ROMS_GPU_NO_GRAPH=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$TAG -o run -- python $R/bench.py --no-cpu-baseline --timing-steps 1 "$@" > $O/kt_$TAG.json 2> $O/kt_$TAG.err || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/kf_$TAG -o run -- python $R/bench.py --no-cpu-baseline --timing-steps 1 "$@" > $O/kf_$TAG.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/kw_$TAG -o run -- python $R/bench.py --no-cpu-baseline --timing-steps 1 "$@" > $O/kw_$TAG.log 2>&1 || exit $?
python3 $R/tools/pmc_kernels.py $(find $O/kf_$TAG -name '*counter_collection.csv') $(find $O/kw_$TAG -name '*counter_collection.csv') \
  --trace $(find $O/kt_$TAG -name '*kernel_trace.csv') > $O/pmck_$TAG.txt
cat $O/pmck_$TAG.txt

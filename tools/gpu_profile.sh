#!/bin/bash
# Kernel-trace profile of the bench plus the two PMC passes (run on the box).
# usage: bash tools/gpu_profile.sh TAG
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- \
  python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_$TAG.json 2> $O/prof_$TAG.err || exit $?
export ROMS_GPU_NO_GRAPH=1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf_$TAG -o run -- \
  python $R/bench.py --steps 2 --warmup 1 --timing-steps 1 --no-cpu-baseline > $O/pmcf_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw_$TAG -o run -- \
  python $R/bench.py --steps 2 --warmup 1 --timing-steps 1 --no-cpu-baseline > $O/pmcw_$TAG.log 2>&1 || exit $?
ls $O/pmcf_$TAG $O/pmcw_$TAG

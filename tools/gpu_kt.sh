#!/bin/bash
# Kernel-trace breakdown of one workload (default C3) on the box.
# usage: bash tools/gpu_kt.sh TAG [c2|c3]
TAG=${1:-kt}; W=${2:-c3}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
M=k_step3d_t_seg; [ $W = c2 ] && M="k_step3d_t_v"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$TAG -o run -- python $R/bench.py --workload $W --steps 5 --warmup 1 --timing-steps 1 --no-cpu-baseline > $O/kt_$TAG.json 2> $O/kt_$TAG.err || { tail -5 $O/kt_$TAG.err; exit 1; }
python3 $R/tools/prof_summary.py $(find $O/kt_$TAG -name "*kernel_trace.csv") --steps 4 --marker $M > $O/kt_$TAG.txt 2>&1
cat $O/kt_$TAG.txt

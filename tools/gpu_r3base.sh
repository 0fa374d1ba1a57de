#!/bin/bash
# Round-3 baseline on the box: default bench line, then C3 kernel trace.
TAG=${1:-r3base}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt3_$TAG -o run -- python $R/bench.py --workload c3 --steps 5 --warmup 1 --timing-steps 1 --no-cpu-baseline > $O/kt3_$TAG.json 2> $O/kt3_$TAG.err || exit 1
python3 $R/tools/prof_summary.py $(find $O/kt3_$TAG -name "*kernel_trace.csv") --steps 4 --marker k_step3d_t_seg > $O/kt3_$TAG.txt 2>&1 || true
echo done

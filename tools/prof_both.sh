# Kernel-trace profiles (rocprofv3 --kernel-trace --stats) of the C2 and C3
# bench commands, with per-step tables.  usage (on the GPU box): bash tools/prof_both.sh TAG
TAG=${1:-x}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2_$TAG -o run -- \
  python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-c3 > $O/prof_c2_$TAG.json 2> $O/prof_c2_$TAG.err || exit 1
python $R/tools/prof_summary.py $O/prof_c2_$TAG/run_kernel_trace.csv --steps 8 --marker "k_step3d_t_h(" > $O/prof_c2_$TAG.txt || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_$TAG -o run -- \
  python $R/bench.py --workload c3 --steps 3 --warmup 1 --timing-steps 1 --no-cpu-baseline > $O/prof_c3_$TAG.json 2> $O/prof_c3_$TAG.err || exit 1
python $R/tools/prof_summary.py $O/prof_c3_$TAG/run_kernel_trace.csv --steps 3 --marker "k_step3d_t_h(" > $O/prof_c3_$TAG.txt || exit 1
head -12 $O/prof_c2_$TAG.txt; head -12 $O/prof_c3_$TAG.txt
echo done

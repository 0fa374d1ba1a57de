#!/bin/bash
# Per-kernel traffic + SQ cycle split of one bench workload (eager steps, no
# graphs): a kernel-trace run, then one rocprofv3 --pmc pass per counter group.
# usage (on the GPU box): bash tools/pmc_all.sh TAG [bench args...]
TAG=${1:-x}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export ROMS_GPU_NO_GRAPH=1
B="python $R/bench.py --no-cpu-baseline --no-c3 --timing-steps 1 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/pa_kt_$TAG -o run -- $B > $O/pa_kt_$TAG.json 2> $O/pa_kt_$TAG.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pa_f_$TAG -o run -- $B > $O/pa_f_$TAG.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pa_w_$TAG -o run -- $B > $O/pa_w_$TAG.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS \
  --output-format csv -d $O/pa_sq_$TAG -o run -- $B > $O/pa_sq_$TAG.log 2>&1 || exit 1
python3 $R/tools/pmc_table.py $(find $O/pa_f_$TAG $O/pa_w_$TAG $O/pa_sq_$TAG -name '*counter_collection.csv') \
  --trace $(find $O/pa_kt_$TAG -name '*kernel_trace.csv') --top 40 > $O/pa_$TAG.txt || exit 1
cat $O/pa_$TAG.txt

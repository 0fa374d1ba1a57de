#!/bin/bash
# Traffic of selected kernels under environment variants (eager steps):
# FETCH_SIZE, WRITE_SIZE, TCC hit/miss passes + kernel trace per variant.
# usage (on the GPU box): bash tools/pmc_ab.sh TAG REGEX "bench args" "ENV=.." ...
TAG=$1; RX=$2; ARGS=$3; shift 3
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export ROMS_GPU_NO_GRAPH=1
n=0
for v in "$@"; do
  n=$((n+1)); D=$O/pab_${TAG}_$n; mkdir -p $D
  for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    env $v timeout -s KILL 300 rocprofv3 --pmc $pass --kernel-include-regex "$RX" --output-format csv -d $D/p$(echo $pass | cut -c1-5) -o run -- \
      python $R/bench.py --no-cpu-baseline --no-c3 --timing-steps 1 $ARGS > $D/log.txt 2>&1 || { tail -5 $D/log.txt; exit 1; }
  done
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex "$RX" --output-format csv -d $D/kt -o run -- \
      python $R/bench.py --no-cpu-baseline --no-c3 --timing-steps 1 $ARGS > $D/log.txt 2>&1 || { tail -5 $D/log.txt; exit 1; }
  echo "== $v"
  python3 $R/tools/pmc_table.py $(find $D -name '*counter_collection.csv') --trace $(find $D/kt -name '*kernel_trace.csv') --top 12
done

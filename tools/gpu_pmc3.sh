#!/bin/bash
# PMC passes on the C3 bench (eager steps): L2 hit/miss, fabric requests, per kernel.
# usage: bash tools/gpu_pmc3.sh TAG [ENV=..]
TAG=${1:-p}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export ROMS_GPU_NO_GRAPH=1
for e in "$@"; do export $e; done
n=0
for P in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  n=$((n+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d $O/pm_${TAG}_$n -o run -- python $R/bench.py --workload c3 --steps 1 --warmup 1 --timing-steps 1 --no-cpu-baseline > $O/pm_${TAG}_$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/pm_${TAG}_$n.log; }
done
python3 $R/tools/pmc_generic.py $(find $O/pm_${TAG}_* -name '*counter_collection.csv') > $O/pm_$TAG.txt
cat $O/pm_$TAG.txt

#!/bin/bash
# PMC passes (one rocprofv3 run each) on the bench, eager steps; per-kernel
# means via tools/pmc_generic.py.
# usage: bash tools/gpu_pmc_passes.sh TAG c2|c3 "CTR CTR ..." "CTR ..." ...
TAG=$1; W=$2; shift 2
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export ROMS_GPU_NO_GRAPH=1
if [ $W = c3 ]; then A="--workload c3"; else A="--no-c3"; fi
n=0
for P in "$@"; do
  n=$((n+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $O/pp_${TAG}_$n -o run -- python $R/bench.py $A --steps 1 --warmup 1 --timing-steps 1 --no-cpu-baseline > $O/pp_${TAG}_$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/pp_${TAG}_$n.log; exit 1; }
done
python3 $R/tools/pmc_generic.py $(find $O/pp_${TAG}_* -name '*counter_collection.csv') > $O/pp_$TAG.txt
cat $O/pp_$TAG.txt

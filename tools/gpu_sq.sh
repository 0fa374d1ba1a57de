#!/bin/bash
# SQ stall breakdown per kernel (one PMC pass, eager launches)
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export ROMS_GPU_NO_GRAPH=1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d $O/sq_$TAG -o run -- \
  python $R/bench.py --steps 2 --warmup 1 --timing-steps 1 --no-cpu-baseline > $O/sq_$TAG.log 2>&1
echo rc=$?
tail -3 $O/sq_$TAG.log

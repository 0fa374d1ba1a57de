#!/bin/bash
# Issue/wait split of every kernel of one workload (c2 | c3, default c2):
# two --pmc passes (SQ cycle buckets + instruction counts), one table
# (tools/pmc_table.py: WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY as % of
# WAVE_CYCLES, instructions per wave).  usage: bash tools/pmc_stall.sh [c2|c3] [TAG]
W=${1:-c2}; TAG=${2:-$W}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export ROMS_GPU_NO_GRAPH=1
S=3; [ $W = c3 ] && S=2
B="python $R/bench.py --no-cpu-baseline --no-secondary --workload $W --timing-steps 1 --steps $S --warmup 1"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/pst1_$TAG -o run -- $B > $O/pst1_$TAG.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS --output-format csv -d $O/pst2_$TAG -o run -- $B > $O/pst2_$TAG.log 2>&1 || exit 1
python3 $R/tools/pmc_table.py $(find $O/pst1_$TAG $O/pst2_$TAG -name '*counter_collection.csv') > $O/pst_$TAG.txt 2>&1
head -40 $O/pst_$TAG.txt

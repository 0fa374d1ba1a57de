#!/bin/bash
# SQ cycle split + traffic of kernels matching REGEX on one bench workload.
# usage (on the GPU box): bash tools/pmc_sq.sh TAG REGEX [bench args...]
TAG=$1; RX=$2; shift 2
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; D=$O/psq_$TAG; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
export ROMS_GPU_NO_GRAPH=1
B="python $R/bench.py --no-cpu-baseline --no-c3 --timing-steps 1 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex "$RX" --output-format csv -d $D/kt -o run -- $B > $D/log 2>&1 || exit 1
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES"; do
  n=$(echo $pass | cut -c1-6)
  timeout -s KILL 300 rocprofv3 --pmc $pass --kernel-include-regex "$RX" --output-format csv -d $D/p_$n -o run -- $B > $D/log 2>&1 || { tail -3 $D/log; exit 1; }
done
python3 $R/tools/pmc_table.py $(find $D -name '*counter_collection.csv') --trace $(find $D/kt -name '*kernel_trace.csv') --top 20
python3 - $D <<'PY'
import csv, collections, glob, sys
v = collections.defaultdict(lambda: collections.defaultdict(float)); c = collections.defaultdict(lambda: collections.defaultdict(int))
for p in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("roms::", "").replace("void ", "")
        v[k][r["Counter_Name"]] += float(r["Counter_Value"]); c[k][r["Counter_Name"]] += 1
for k in v:
    m = {n: v[k][n] / c[k][n] for n in v[k]}
    w = m.get("SQ_WAVES", 1)
    print("%-34s " % k[:34] + " ".join("%s=%.0f" % (n.replace("SQ_", "").replace("INSTS_", "I_"), m[n] / w) for n in sorted(m) if n.startswith("SQ_") and n != "SQ_WAVES"))
PY

#!/bin/bash
# SQ busy/stall counters per kernel for one bench workload (eager launches).
# usage: bash tools/gpu_sq2.sh TAG [bench args...]
TAG=${1:-x}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export ROMS_GPU_NO_GRAPH=1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVES --output-format csv -d $O/sq_$TAG -o run -- \
  python $R/bench.py --steps 1 --warmup 1 --timing-steps 1 --no-cpu-baseline "$@" > $O/sq_$TAG.log 2>&1 || exit $?
python3 - $O/sq_$TAG <<'PY' > $O/sq_$TAG.txt
import csv, glob, sys, collections
p = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in csv.DictReader(open(p)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("roms::", "")
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES": cnt[k] += 1
print("%-34s %6s %9s %7s %7s %7s %7s %9s %8s" % ("kernel", "calls", "waves", "wait%", "winst%", "valu%", "any%", "valu/wave", "vmem/wv"))
for k, c in sorted(agg.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"]):
    wc = c["SQ_WAVE_CYCLES"] or 1
    w = c["SQ_WAVES"] or 1
    print("%-34s %6d %9.0f %7.1f %7.1f %7.1f %7.1f %9.0f %8.0f" % (k[:34], cnt[k], w / max(cnt[k], 1), 100 * c["SQ_WAIT_ANY"] / wc,
          100 * c["SQ_WAIT_INST_ANY"] / wc, 100 * c["SQ_ACTIVE_INST_VALU"] / wc, 100 * c["SQ_ACTIVE_INST_ANY"] / wc,
          c["SQ_INSTS_VALU"] / w, c["SQ_INSTS_VMEM"] / w))
PY
cat $O/sq_$TAG.txt | head -30

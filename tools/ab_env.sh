#!/bin/bash
# A/B of environment switches on one bench workload: per variant, the per-step
# time and the routine table.  usage (on the GPU box):
#   bash tools/ab_env.sh TAG "bench args" "ENV=.. ENV2=.." "ENV=.." ...
TAG=$1; ARGS=$2; shift 2
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
n=0
for v in "$@"; do
  n=$((n+1))
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-c3 $ARGS > $O/ab_${TAG}_$n.json 2> $O/ab_${TAG}_$n.err || { tail -20 $O/ab_${TAG}_$n.err; exit 1; }
  python3 - "$O/ab_${TAG}_$n.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["routines"]
print("%-40s %7.2f ms/step | " % (sys.argv[2], d["ms_per_step"]) + " ".join("%s=%.3f" % (k, v["ms_per_call"]) for k, v in r.items()))
PY
done

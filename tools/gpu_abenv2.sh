#!/bin/bash
# C2 A/B of environment switches on the current library (optional parity tests first).
# usage: bash tools/gpu_abenv2.sh TAG "pytest -k expr" "ENV=.." "ENV=.." ...
TAG=$1; K=$2; shift 2
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/t_$TAG.log 2>&1 || { echo TESTFAIL; tail -30 $O/t_$TAG.log; exit 1; }
  tail -1 $O/t_$TAG.log
fi
n=0
for v in "$@"; do
  n=$((n+1))
  env $v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --timing-steps 3 --no-cpu-baseline --no-c3 > $O/ab2_${TAG}_$n.json 2> $O/ab2_${TAG}_$n.err || { tail -20 $O/ab2_${TAG}_$n.err; exit 1; }
  python3 - "$O/ab2_${TAG}_$n.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["routines"]
print("%-28s %7.3f ms/step | " % (sys.argv[2], d["ms_per_step"]) + " ".join("%s=%.3f" % (k, v["ms_per_call"]) for k, v in r.items()))
PY
done

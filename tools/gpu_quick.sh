#!/bin/bash
# Quick GPU iteration: selected parity tests, then the C2+C3 bench with and
# without an A/B switch.  usage: bash tools/gpu_quick.sh TAG "pytest -k expr" "ENV=1"
TAG=${1:-x}; K=${2:-}; AB=${3:-}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/q_$TAG.log 2>&1 || { tail -40 $O/q_$TAG.log; exit 1; }
  tail -2 $O/q_$TAG.log
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/qb_$TAG.json 2> $O/qb_$TAG.err || { tail -20 $O/qb_$TAG.err; exit 1; }
if [ -n "$AB" ]; then
  env $AB timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/qb_${TAG}_ab.json 2> $O/qb_${TAG}_ab.err || { tail -20 $O/qb_${TAG}_ab.err; exit 1; }
fi
python3 - $O/qb_$TAG.json $O/qb_${TAG}_ab.json <<'PY'
import json, sys, os
for p in sys.argv[1:]:
    if not os.path.exists(p): continue
    d = json.load(open(p))
    for name, w in (("C2", d), ("C3", d.get("c3"))):
        if not w: continue
        r = w["routines"]
        print(os.path.basename(p), name, "%.3f ms/step" % w["ms_per_step"], " ".join("%s=%.3f" % (k, v["ms_per_step"]) for k, v in r.items()))
PY

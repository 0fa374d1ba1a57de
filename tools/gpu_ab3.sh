#!/bin/bash
# Seg-solver parity tests on the new library, then C3 A/B: base (HEAD build) vs new.
TAG=${1:-ab}; K=${2:-"colseg or c3_ or uv2_fused or chain"}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/t_$TAG.log 2>&1 || { echo TESTFAIL; tail -30 $O/t_$TAG.log; exit 1; }
tail -1 $O/t_$TAG.log
for v in base new base new; do
  if [ $v = base ]; then L=$R/ucla-roms_amd/libromsgpu_base.so; else L=$R/ucla-roms_amd/libromsgpu.so; fi
  ROMS_GPU_LIB=$L timeout -k 10 300 python bench.py --workload c3 --steps 5 --warmup 2 --timing-steps 2 --no-cpu-baseline > $O/ab_${TAG}_$v.json 2> $O/ab_${TAG}_$v.err || { tail -20 $O/ab_${TAG}_$v.err; exit 1; }
  python3 - "$O/ab_${TAG}_$v.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["routines"]
print("%-6s %7.2f ms/step | " % (sys.argv[2], d["ms_per_step"]) + " ".join("%s=%.3f" % (k, v["ms_per_call"]) for k, v in r.items()))
PY
done

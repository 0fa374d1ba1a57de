#!/bin/bash
# A/B of library builds (ucla-roms_amd/libromsgpu_<tag>.so, "cur" = the
# in-tree build): parity tests selected by -k on each, then the bench.
# usage: bash tools/gpu_ablib.sh TAG WORKLOAD(c2|c3) "pytest -k expr" tag1 tag2 ...
TAG=$1; W=$2; K=$3; shift 3
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
lib() { if [ "$1" = cur ]; then echo $R/ucla-roms_amd/libromsgpu.so; else echo $R/ucla-roms_amd/libromsgpu_$1.so; fi; }
if [ -n "$K" ]; then
  for v in $(echo "$@" | tr ' ' '\n' | sort -u); do
    ROMS_GPU_LIB=$(lib $v) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/t_${TAG}_$v.log 2>&1 || { echo TESTFAIL $v; tail -30 $O/t_${TAG}_$v.log; exit 1; }
    echo "$v: $(tail -1 $O/t_${TAG}_$v.log)"
  done
fi
n=0
for v in "$@"; do
  n=$((n+1))
  if [ $W = c3 ]; then A="--workload c3 --steps 5 --warmup 2 --timing-steps 2"; else A="--steps 20 --warmup 3 --timing-steps 3 --no-c3"; fi
  ROMS_GPU_LIB=$(lib $v) timeout -k 10 300 python bench.py $A --no-cpu-baseline > $O/abl_${TAG}_$n.json 2> $O/abl_${TAG}_$n.err || { tail -20 $O/abl_${TAG}_$n.err; exit 1; }
  python3 - "$O/abl_${TAG}_$n.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["routines"]
print("%-8s %7.2f ms/step | " % (sys.argv[2], d["ms_per_step"]) + " ".join("%s=%.3f" % (k, v["ms_per_call"]) for k, v in r.items()))
PY
done

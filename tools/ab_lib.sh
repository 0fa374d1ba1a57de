#!/bin/bash
# A/B of library builds (tools/build_variant.sh) on one bench workload, after
# the segment-solver parity tests of each variant.
# usage (on the GPU box): bash tools/ab_lib.sh TAG "bench args" "pytest -k expr" lib1 lib2 ...
#   lib "base" = ucla-roms_amd/libromsgpu.so, otherwise ucla-roms_amd/libromsgpu_<lib>.so
TAG=$1; ARGS=$2; K=$3; shift 3
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for v in "$@"; do
  if [ "$v" = base ]; then L=$R/ucla-roms_amd/libromsgpu.so; else L=$R/ucla-roms_amd/libromsgpu_$v.so; fi
  if [ -n "$K" ]; then
    ROMS_GPU_LIB=$L timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/abl_${TAG}_$v.log 2>&1 || { echo "$v TESTFAIL"; tail -30 $O/abl_${TAG}_$v.log; exit 1; }
    echo "$v: $(tail -1 $O/abl_${TAG}_$v.log)"
  fi
  ROMS_GPU_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-c3 $ARGS > $O/abl_${TAG}_$v.json 2> $O/abl_${TAG}_$v.err || { tail -20 $O/abl_${TAG}_$v.err; exit 1; }
  python3 - "$O/abl_${TAG}_$v.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["routines"]
print("%-10s %7.2f ms/step | " % (sys.argv[2], d["ms_per_step"]) + " ".join("%s=%.3f" % (k, v["ms_per_call"]) for k, v in r.items()))
PY
done

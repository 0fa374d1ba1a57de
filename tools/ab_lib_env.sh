#!/bin/bash
# A/B of (library build, environment) pairs on one bench workload.
# usage (on the GPU box): bash tools/ab_lib_env.sh TAG "bench args" "lib|ENV=.. ENV2=.." ...
#   lib "base" = ucla-roms_amd/libromsgpu.so, otherwise ucla-roms_amd/libromsgpu_<lib>.so
TAG=$1; ARGS=$2; shift 2
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
n=0
for v in "$@"; do
  n=$((n+1)); lib=${v%%|*}; envs=${v#*|}
  if [ "$lib" = base ]; then L=$R/ucla-roms_amd/libromsgpu.so; else L=$R/ucla-roms_amd/libromsgpu_$lib.so; fi
  env ROMS_GPU_LIB=$L $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-c3 $ARGS > $O/abe_${TAG}_$n.json 2> $O/abe_${TAG}_$n.err || { tail -20 $O/abe_${TAG}_$n.err; exit 1; }
  python3 - "$O/abe_${TAG}_$n.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["routines"]
print("%-36s %7.2f ms/step | " % (sys.argv[2], d["ms_per_step"]) + " ".join("%s=%.3f" % (k, v["ms_per_call"]) for k, v in r.items()))
PY
done

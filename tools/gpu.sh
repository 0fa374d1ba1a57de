#!/bin/bash
# Every GPU-box job of this repository, parameterised (run on the box from the
# repo root, e.g. gpurun -- 'bash tools/gpu.sh suite r4_a'); outputs go to
# gpurun_out/.  Each GPU step has its own time limit and the first failure
# ends the job.
#   suite TAG                 full `-m gpu` suite, smoke(), the default bench line
#   tests TAG ARGS...         selected tests (pytest arguments)
#   bench TAG [BENCH ARGS]    one bench line
#   trace TAG c2|c3           rocprofv3 --kernel-trace --stats of the bench, per-step kernel table
#   pmc                       PMC traffic tables (one --pmc pass per counter; profiles/pmc_traffic*.json)
#   ab TAG c2|c3 KEXPR V...   A/B of variants, same box back to back: parity tests selected by the
#                             pytest -k expression KEXPR (empty: none) on each, then the bench line.
#                             V = lib:<tag> (ucla-roms_amd/libromsgpu_<tag>.so from tools/build_variant.sh;
#                             lib:cur the in-tree build) or env:VAR=1,VAR2=0 (environment switches)
#   stall                     issue/wait PMC of the C2 kernels (tools/pmc_stall.sh)
#   valu TAG                  VALU instruction mix per C3 kernel (tools/pmc_valu.py -> gpurun_out/pmc_valu_c3.json)
#   final TAG 1|2             1: the default bench line, C3/C2 kernel traces; 2: PMC traffic and VALU
#                             tables and a 2-rank one-GPU rehearsal (both exchange orders)
CMD=$1; TAG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
row() {   # one line per bench json: ms/step and the routine table
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["routines"]
print("%-28s %7.2f ms/step | " % (sys.argv[2], d["ms_per_step"]) + " ".join("%s=%.3f" % (k, v["ms_per_call"]) for k, v in r.items()))
PY
}
wargs() { if [ "$1" = c3 ]; then echo "--workload c3 --steps 5 --warmup 2 --timing-steps 2"; else echo "--workload c2 --steps 20 --warmup 3 --timing-steps 3 --no-secondary"; fi; }
case $CMD in
suite)
  timeout -k 10 1500 $PYT -v -rf tests -m gpu -x > $O/tests_$TAG.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests_$TAG.log; exit 1; }
  tail -1 $O/tests_$TAG.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke_$TAG.log; exit 1; }
  tail -1 $O/smoke_$TAG.log
  timeout -k 10 500 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo BENCHFAIL; tail -20 $O/bench_$TAG.err; exit 1; }
  row $O/bench_$TAG.json bench ;;
tests)
  timeout -k 10 1100 $PYT -v -rf -s "$@" > $O/tests_$TAG.log 2>&1; rc=$?
  tail -3 $O/tests_$TAG.log; exit $rc ;;
bench)
  timeout -k 10 600 python bench.py "$@" > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo BENCHFAIL; tail -20 $O/bench_$TAG.err; exit 1; }
  row $O/bench_$TAG.json "$TAG" ;;
trace)
  W=${1:-c3}; M=k_step3d_t_seg; [ $W = c2 ] && M=k_step3d_t_v
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$TAG -o run -- python $R/bench.py --workload $W --steps 5 --warmup 1 --timing-steps 1 --no-cpu-baseline --no-secondary > $O/kt_$TAG.json 2> $O/kt_$TAG.err || { tail -5 $O/kt_$TAG.err; exit 1; }
  python3 $R/tools/prof_summary.py $(find $O/kt_$TAG -name "*kernel_trace.csv") --steps 4 --marker $M > $O/kt_$TAG.txt 2>&1
  head -30 $O/kt_$TAG.txt ;;
pmc)
  cd /tmp && export TMPDIR=/tmp
  export ROMS_GPU_NO_GRAPH=1
  for W in c2 c3; do
    if [ $W = c2 ]; then B="python $R/bench.py --no-cpu-baseline --no-secondary --workload c2 --timing-steps 1 --steps 4 --warmup 1"; M=k_step3d_t_v
    else B="python $R/bench.py --no-cpu-baseline --no-secondary --workload c3 --timing-steps 1 --steps 2 --warmup 1"; M=k_step3d_t_segb; fi
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pt_f_$W -o run -- $B > $O/pt_f_$W.log 2>&1 || exit 1
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pt_w_$W -o run -- $B > $O/pt_w_$W.log 2>&1 || exit 1
    python3 $R/tools/pmc_traffic.py $(find $O/pt_f_$W -name '*counter_collection.csv') $(find $O/pt_w_$W -name '*counter_collection.csv') \
      --steps-marker $M --nfast 82 --out $O/pmc_traffic_$W.json || exit 1
  done
  echo pmc done ;;
ab)
  W=$1; K=$2; shift 2
  for v in "$@"; do
    case $v in
      lib:cur) E="ROMS_GPU_LIB=$R/ucla-roms_amd/libromsgpu.so" ;;
      lib:*) E="ROMS_GPU_LIB=$R/ucla-roms_amd/libromsgpu_${v#lib:}.so" ;;
      env:*) E=$(echo "${v#env:}" | tr ',' ' ') ;;
      *) echo "bad variant $v"; exit 2 ;;
    esac
    n=$(echo "$v" | tr -c 'A-Za-z0-9_' '_')
    if [ -n "$K" ]; then
      env $E timeout -k 10 900 $PYT tests -m gpu -x -k "$K" > $O/ab_${TAG}_$n.log 2>&1 || { echo "$v TESTFAIL"; tail -30 $O/ab_${TAG}_$n.log; exit 1; }
      echo "$v: $(tail -1 $O/ab_${TAG}_$n.log)"
    fi
  done
  for v in "$@"; do
    case $v in
      lib:cur) E="ROMS_GPU_LIB=$R/ucla-roms_amd/libromsgpu.so" ;;
      lib:*) E="ROMS_GPU_LIB=$R/ucla-roms_amd/libromsgpu_${v#lib:}.so" ;;
      env:*) E=$(echo "${v#env:}" | tr ',' ' ') ;;
    esac
    n=$(echo "$v" | tr -c 'A-Za-z0-9_' '_')
    env $E timeout -k 10 400 python bench.py $(wargs $W) --no-cpu-baseline > $O/ab_${TAG}_$n.json 2> $O/ab_${TAG}_$n.err || { echo "$v BENCHFAIL"; tail -20 $O/ab_${TAG}_$n.err; exit 1; }
    row $O/ab_${TAG}_$n.json "$v"
  done ;;
stall)
  bash $R/tools/pmc_stall.sh ;;
valu)
  # VALU instruction mix per kernel at C3 (one --pmc pass of 8 SQ counters)
  cd /tmp && export TMPDIR=/tmp
  export ROMS_GPU_NO_GRAPH=1
  B="python $R/bench.py --no-cpu-baseline --no-secondary --workload c3 --timing-steps 1 --steps 2 --warmup 1"
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 --output-format csv -d $O/pv_$TAG -o run -- $B > $O/pv_$TAG.log 2>&1 || exit 1
  python3 $R/tools/pmc_valu.py $(find $O/pv_$TAG -name '*counter_collection.csv') --out $O/pmc_valu_c3.json || exit 1 ;;
final)
  # the round's profile set in two calls (each within gpurun's limit):
  # final TAG 1 = bench line + C3/C2 kernel traces; final TAG 2 = PMC traffic
  # and VALU tables + the 2-rank one-GPU rehearsal
  PART=${1:-1}
  if [ "$PART" = 1 ]; then
    timeout -k 10 500 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo BENCHFAIL; tail -20 $O/bench_$TAG.err; exit 1; }
    row $O/bench_$TAG.json bench
    bash $R/tools/gpu.sh trace ${TAG}_c3 c3 || exit 1
    bash $R/tools/gpu.sh trace ${TAG}_c2 c2 || exit 1
  else
    bash $R/tools/gpu.sh pmc x || exit 1
    bash $R/tools/gpu.sh valu $TAG || exit 1
    cd $R
    timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline --no-secondary > $O/bench_${TAG}_n2.json 2> $O/bench_${TAG}_n2.err || { tail -10 $O/bench_${TAG}_n2.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${TAG}_n2.json')); print('n2', d['ms_per_step'], d['config'].get('exchange_overlap'))"
  fi ;;
*) echo "usage: bash tools/gpu.sh suite|tests|bench|trace|pmc|ab|stall|final TAG ..."; exit 2 ;;
esac

# Parity suite + C2/C3 benches without the CPU baseline (quick A/B of a kernel change).
# usage (on the GPU box): bash tools/quick.sh TAG [extra env for the benches]
TAG=${1:-x}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests_$TAG.log; exit 1; }
tail -1 $O/tests_$TAG.log
env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/q2_$TAG.json 2> $O/q2_$TAG.err || { tail -20 $O/q2_$TAG.err; exit 1; }
env "$@" timeout -k 10 300 python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/q3_$TAG.json 2> $O/q3_$TAG.err || { tail -20 $O/q3_$TAG.err; exit 1; }
python -c "
import json
for w in ('q2','q3'):
    d=json.load(open('$O/%s_$TAG.json'%w)); print(w, round(d['ms_per_step'],3), {k:round(v['ms_per_call'],3) for k,v in d['routines'].items()})
"

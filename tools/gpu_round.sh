#!/bin/bash
# Full GPU round trip on the box: parity tests, C2 bench (+cpu baseline), C3
# bench, then the newest test file(s) given as extra args (no -x).
# usage: bash tools/gpu_round.sh TAG [new_test_file ...]
TAG=${1:-x}; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
IGN=""
for f in "$@"; do IGN="$IGN --ignore=$f"; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $IGN > $O/tests_$TAG.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests_$TAG.log; exit 1; }
tail -2 $O/tests_$TAG.log
timeout -k 10 300 python bench.py > $O/bench_c2_$TAG.json 2> $O/bench_c2_$TAG.err || { echo BENCHFAIL; tail -20 $O/bench_c2_$TAG.err; exit 1; }
timeout -k 10 400 python bench.py --workload c3 --steps 5 --warmup 2 > $O/bench_c3_$TAG.json 2> $O/bench_c3_$TAG.err || { echo C3FAIL; tail -20 $O/bench_c3_$TAG.err; exit 1; }
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -v --timeout 300 --timeout-method thread > $O/tests_new_$TAG.log 2>&1
  echo "new tests rc=$?"; tail -15 $O/tests_new_$TAG.log
fi
echo done

#!/bin/bash
# Full GPU suite, smoke and the default bench line from this tree (no traces).
# usage (on the GPU box): bash tools/gpu_suite.sh TAG
TAG=${1:-suite}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests_$TAG.log; exit 1; }
tail -1 $O/tests_$TAG.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke_$TAG.log; exit 1; }
tail -1 $O/smoke_$TAG.log
timeout -k 10 500 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo BENCHFAIL; tail -20 $O/bench_$TAG.err; exit 1; }
echo bench done

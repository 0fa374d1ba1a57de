#!/bin/bash
# Round-end refresh on the box: full GPU suite, smoke, default bench line,
# C2/C3 kernel traces and the PMC traffic tables, all from this tree.
# usage: bash tools/gpu_final.sh TAG
TAG=${1:-final}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests_$TAG.log; exit 1; }
tail -1 $O/tests_$TAG.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke_$TAG.log; exit 1; }
tail -1 $O/smoke_$TAG.log
timeout -k 10 500 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo BENCHFAIL; tail -20 $O/bench_$TAG.err; exit 1; }
echo bench done
bash tools/gpu_kt.sh ${TAG}c3 c3 > /dev/null || { echo KT3FAIL; exit 1; }
bash tools/gpu_kt.sh ${TAG}c2 c2 > /dev/null || { echo KT2FAIL; exit 1; }
echo traces done
bash tools/gpu_pmc_traffic.sh > $O/pmc_$TAG.log 2>&1 || { echo PMCFAIL; tail -10 $O/pmc_$TAG.log; exit 1; }
echo all done

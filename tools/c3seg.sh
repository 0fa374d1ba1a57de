# A/B of the segment-partitioned column solvers on C3 (1024x1024x100, 1 GPU):
# default (colseg for N > 63) vs the sequential solvers with global scratch.
# usage (on the GPU box): bash tools/c3seg.sh TAG
TAG=${1:-x}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_colseg.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/colseg_$TAG.log 2>&1 || { tail -30 $O/colseg_$TAG.log; exit 1; }
tail -3 $O/colseg_$TAG.log
timeout -k 10 300 python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3seg_on_$TAG.json 2> $O/c3seg_on_$TAG.err || exit 1
ROMS_GPU_COLSEG=0 timeout -k 10 300 python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3seg_off_$TAG.json 2> $O/c3seg_off_$TAG.err || exit 1
echo done

# A/B of the segment-partitioned column solvers on C2 (N = 50): forced on vs
# the default sequential LDS solvers.  usage (on the GPU box): bash tools/c2seg.sh TAG
TAG=${1:-x}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
ROMS_GPU_COLSEG=1 timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/c2seg_on_$TAG.json 2> $O/c2seg_on_$TAG.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/c2seg_off_$TAG.json 2> $O/c2seg_off_$TAG.err || exit 1
echo done

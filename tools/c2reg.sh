# Register-resident column solvers at C2 (N = 50): parity, then A/B against
# the two-slot LDS form.  usage (on the GPU box): bash tools/c2reg.sh TAG
TAG=${1:-x}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_colseg.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/reg_$TAG.log 2>&1 || { tail -30 $O/reg_$TAG.log; exit 1; }
tail -3 $O/reg_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/c2reg_on_$TAG.json 2> $O/c2reg_on_$TAG.err || exit 1
ROMS_GPU_COLREG=0 timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/c2reg_off_$TAG.json 2> $O/c2reg_off_$TAG.err || exit 1
echo done

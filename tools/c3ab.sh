R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_base.json 2> $O/c3_base.err || exit 1
ROMS_GPU_COL_GLOBAL=0 timeout -k 10 300 python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_lds.json 2> $O/c3_lds.err || exit 1
ROMS_GPU_COL_GLOBAL=0 ROMS_GPU_COLSEG=0 timeout -k 10 300 python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_lds_noseg.json 2> $O/c3_lds_noseg.err || exit 1

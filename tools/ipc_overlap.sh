# Fast-loop overlap with the IPC transport (one GPU, every exchange through it).
# usage (on the GPU box): bash tools/ipc_overlap.sh TAG
TAG=${1:-x}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 ROMS_BENCH_FORCE_COMM=1
MASTER_PORT=29641 ROMS_GPU_S2D_OVERLAP=1 timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/iov_on_$TAG.json 2> $O/iov_on_$TAG.err || { tail -20 $O/iov_on_$TAG.err; exit 1; }
MASTER_PORT=29642 timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/iov_off_$TAG.json 2> $O/iov_off_$TAG.err || { tail -20 $O/iov_off_$TAG.err; exit 1; }
python -c "
import json
for w in ('on','off'):
    d=json.load(open('$O/iov_%s_$TAG.json'%w)); print(w, round(d['ms_per_step'],3), d['config']['halo_transport'])
"

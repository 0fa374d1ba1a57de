# IPC halo transport: full GPU test suite, then the one-GPU multi-rank bench
# (every exchange through the transport) with IPC and with RCCL.
# usage (on the GPU box): bash tools/ipc.sh TAG
TAG=${1:-x}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests_$TAG.log; exit 1; }
tail -1 $O/tests_$TAG.log
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 ROMS_BENCH_FORCE_COMM=1
MASTER_PORT=29631 timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/ipc_on_$TAG.json 2> $O/ipc_on_$TAG.err || { tail -20 $O/ipc_on_$TAG.err; exit 1; }
MASTER_PORT=29633 ROMS_GPU_HALO_IPC_FUSED=0 timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/ipc_sep_$TAG.json 2> $O/ipc_sep_$TAG.err || exit 1
MASTER_PORT=29632 ROMS_GPU_HALO_IPC=0 timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/ipc_off_$TAG.json 2> $O/ipc_off_$TAG.err || { tail -20 $O/ipc_off_$TAG.err; exit 1; }
python -c "
import json
for w in ('on','sep','off'):
    d=json.load(open('$O/ipc_%s_$TAG.json'%w)); print(w, round(d['ms_per_step'],3), d['config']['halo_transport'], round(d['routines']['step2d']['ms_per_call'],4))
"
echo done

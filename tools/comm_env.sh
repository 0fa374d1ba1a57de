# RCCL tuning sweep for the halo exchanges (every exchange routed through
# RCCL, self-addressed, on one GPU).  usage (on the GPU box): bash tools/comm_env.sh TAG
TAG=${1:-x}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 ROMS_BENCH_FORCE_COMM=1
run() {  # name port env...
  local n=$1 p=$2; shift 2
  env MASTER_PORT=$p "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/ce_${n}_$TAG.json 2> $O/ce_${n}_$TAG.err || { tail -5 $O/ce_${n}_$TAG.err; return 1; }
  python -c "import json;d=json.load(open('$O/ce_${n}_$TAG.json'));print('$n',round(d['ms_per_step'],3))"
}
run base 29601 && run llthr 29602 NCCL_P2P_LL_THRESHOLD=1048576 && run protoLL 29603 NCCL_PROTO=LL && run ll128 29604 NCCL_PROTO=LL128 && run ch1 29605 NCCL_MAX_NCHANNELS=1 && run llch 29606 NCCL_PROTO=LL NCCL_MAX_NCHANNELS=2
echo done

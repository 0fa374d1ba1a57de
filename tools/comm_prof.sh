# Cost of the multi-rank exchange path on one GPU: bench with every halo
# exchange routed through RCCL (self-addressed), plain and under a kernel
# trace.  usage (on the GPU box): bash tools/comm_prof.sh TAG
TAG=${1:-x}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 ROMS_BENCH_FORCE_COMM=1
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/comm_$TAG.json 2> $O/comm_$TAG.err || { tail -20 $O/comm_$TAG.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
MASTER_PORT=29518 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/commprof_$TAG -o run -- python $R/bench.py --steps 5 --warmup 2 --timing-steps 1 --no-cpu-baseline > $O/commprof_$TAG.json 2> $O/commprof_$TAG.err || { tail -20 $O/commprof_$TAG.err; exit 1; }
echo done

#!/bin/bash
# profiles/pmc_traffic.json (C2, the bench default) and pmc_traffic_c3.json
# from the committed kernels: eager steps, one rocprofv3 --pmc pass per counter.
# usage (on the GPU box): bash tools/gpu_pmc_traffic.sh
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export ROMS_GPU_NO_GRAPH=1
for W in c2 c3; do
  if [ $W = c2 ]; then B="python $R/bench.py --no-cpu-baseline --no-c3 --timing-steps 1 --steps 4 --warmup 1"; M=k_step3d_t_v; N=82
  else B="python $R/bench.py --no-cpu-baseline --no-c3 --workload c3 --timing-steps 1 --steps 2 --warmup 1"; M=k_step3d_t_seg; N=82; fi
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pt_f_$W -o run -- $B > $O/pt_f_$W.log 2>&1 || exit 1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pt_w_$W -o run -- $B > $O/pt_w_$W.log 2>&1 || exit 1
  OUT=$O/pmc_traffic_$W.json
  python3 $R/tools/pmc_traffic.py $(find $O/pt_f_$W -name '*counter_collection.csv') $(find $O/pt_w_$W -name '*counter_collection.csv') \
    --steps-marker $M --nfast $N --out $OUT || exit 1
done
echo done

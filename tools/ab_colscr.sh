set -o pipefail
mkdir -p gpurun_out
ROMS_GPU_COL_GLOBAL=1 timeout -k 10 400 python -m pytest tests/test_gpu_parity.py tests/test_gpu_lmd.py -x -q -m gpu > gpurun_out/colglb_tests.log 2>&1 || { echo TESTFAIL; tail -20 gpurun_out/colglb_tests.log; exit 1; }
tail -2 gpurun_out/colglb_tests.log
timeout -k 10 300 python bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c3_glb.json 2>/dev/null
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c2_lds.json 2>/dev/null
ROMS_GPU_COL_GLOBAL=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c2_glb.json 2>/dev/null
echo done

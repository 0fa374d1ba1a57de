set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ipc.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_ipc.log 2>&1 || { tail -50 gpurun_out/r2_ipc.log; exit 1; }
tail -8 gpurun_out/r2_ipc.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_t2.log 2>&1 || { tail -30 gpurun_out/r2_t2.log; exit 1; }
tail -3 gpurun_out/r2_t2.log
timeout -k 10 400 python bench.py > gpurun_out/r2_bench_a.json 2> gpurun_out/r2_bench_a.err || { tail -30 gpurun_out/r2_bench_a.err; exit 1; }
head -c 1500 gpurun_out/r2_bench_a.json
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 --no-c3 > gpurun_out/r2_bench_n2.json 2> gpurun_out/r2_bench_n2.err || { tail -30 gpurun_out/r2_bench_n2.err; exit 1; }
head -c 800 gpurun_out/r2_bench_n2.json

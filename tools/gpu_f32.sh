# fp32 CNN path: GPU tests, then per-step timing (bench.py --dtype fp32 at N=1).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_cnn_f32.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_f32.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --dtype fp32 --scaling weak --steps 100 --warmup 10 > gpurun_out/bench_f32.log 2>&1 || exit 1
echo rc=$?

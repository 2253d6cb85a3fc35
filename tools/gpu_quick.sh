# Quick check after a kernel change: CNN + Linear GPU tests, kbench at B=256, N=1 benches.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/quick.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_cnn_bwd_exact.py tests/test_gpu_linear.py tests/test_gpu_comm.py tests/test_gpu_optim.py -x -q --timeout 120 --timeout-method thread >> gpurun_out/quick.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/kbench.py 256 1024 >> gpurun_out/quick.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/kbench_fc.py >> gpurun_out/quick.log 2>&1 || exit 1
timeout -k 10 120 python bench.py >> gpurun_out/quick.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --model linear >> gpurun_out/quick.log 2>&1 || exit 1
echo rc=$?

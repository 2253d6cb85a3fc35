set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cnn_bwd_exact.py tests/test_gpu_cnn.py tests/test_gpu_optim.py > gpurun_out/t_cnn.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/kbench.py 256 1024 8192 > gpurun_out/kbench.log 2>&1
echo rc=$?

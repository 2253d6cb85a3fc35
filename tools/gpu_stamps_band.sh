set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_cnn_bwd_exact.py tests/test_gpu_linear.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_cnn.log 2>&1 || exit 1
: > gpurun_out/stamps_band.log
for B in 32 64 128; do PDM_EXT_PATH=build/stamps/_C.cpython-310-x86_64-linux-gnu.so timeout -k 10 120 python -u tools/stamps_band.py $B >> gpurun_out/stamps_band.log 2>&1 || exit 1; done
echo rc=$?

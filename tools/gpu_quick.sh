# Quick check after a kernel change: CNN GPU tests (fp64-exact backward, end to end,
# N>1 chain), kbench at the strong-scaling batches + B=256/1024, N=1 bench (weak + FORCE_COMM).
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/quick.log
: > $L
timeout -k 10 400 python -u -m pytest tests/test_gpu_cnn_bwd_exact.py tests/test_gpu_cnn.py tests/test_gpu_comm.py -x -q --timeout 120 --timeout-method thread >> $L 2>&1 || exit 1
timeout -k 10 300 python -u tools/kbench.py 32 64 128 256 1024 >> $L 2>&1 || exit 1
timeout -k 10 300 python -u tools/kbench.py 256 >> $L 2>&1 || exit 1
timeout -k 10 120 python bench.py --scaling weak >> $L 2>&1 || exit 1
PDM_FORCE_COMM=1 timeout -k 10 200 python bench.py --scaling weak >> $L 2>&1 || exit 1
PDM_EXT_PATH=build/stamps/_C.cpython-310-x86_64-linux-gnu.so timeout -k 10 120 python -u tools/stamps.py 256 >> $L 2>&1 || exit 1
echo rc=$?

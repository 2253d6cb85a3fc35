# Quick check after a kernel change: CNN GPU tests (fp64-exact backward, end to end,
# N>1 chain), kbench at the strong-scaling batches, N=1 benches (weak + FORCE_COMM chain).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/quick.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_cnn_bwd_exact.py tests/test_gpu_cnn.py tests/test_gpu_comm.py -x -q --timeout 120 --timeout-method thread >> gpurun_out/quick.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/kbench.py 32 64 128 256 >> gpurun_out/quick.log 2>&1 || exit 1
for B in 32 64 128 256; do
  PDM_FORCE_COMM=1 PDM_COMM=rccl timeout -k 10 120 python bench.py --scaling weak --batch-per-rank $B >> gpurun_out/quick.log 2>&1 || exit 1
  timeout -k 10 120 python bench.py --scaling weak --batch-per-rank $B >> gpurun_out/quick.log 2>&1 || exit 1
done
echo rc=$?

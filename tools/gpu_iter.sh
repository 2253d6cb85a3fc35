# One iteration of the small-batch work: CNN/Linear/comm GPU tests, band stamps, kbench and
# the N=1 benches (local chain and the FORCE_COMM N>1 chain) at the strong-scaling batches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_cnn_bwd_exact.py tests/test_gpu_linear.py tests/test_gpu_comm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_iter.log 2>&1 || exit 1
: > gpurun_out/stamps_band.log
for B in 32 64 128; do PDM_EXT_PATH=build/stamps/_C.cpython-310-x86_64-linux-gnu.so timeout -k 10 120 python -u tools/stamps_band.py $B >> gpurun_out/stamps_band.log 2>&1 || exit 1; done
timeout -k 10 300 python -u tools/kbench.py 32 64 128 256 > gpurun_out/kb_iter.log 2>&1 || exit 1
: > gpurun_out/bench_iter.log
for B in 32 64 128 256; do
  PDM_FORCE_COMM=1 PDM_COMM=rccl timeout -k 10 120 python bench.py --scaling weak --batch-per-rank $B >> gpurun_out/bench_iter.log 2>&1 || exit 1
  timeout -k 10 120 python bench.py --scaling weak --batch-per-rank $B >> gpurun_out/bench_iter.log 2>&1 || exit 1
done
echo rc=$?

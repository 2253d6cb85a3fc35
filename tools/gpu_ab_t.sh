# CNN / comm / bench GPU tests on the in-tree build, the interleaved A/B against $@, then the
# N>1 chain (PDM_FORCE_COMM, every RCCL fc-update placement calibrated) at B = 32 .. 256
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cnn_bwd_exact.py tests/test_gpu_cnn.py tests/test_gpu_comm.py tests/test_gpu_bench.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || exit 1
bash tools/gpu_ab.sh "$@" || exit 1
: > gpurun_out/fc_modes.log
for B in 32 64 128 256; do
  PDM_FORCE_COMM=1 timeout -k 10 300 python bench.py --scaling weak --batch-per-rank $B >> gpurun_out/fc_modes.log 2>&1 || exit 1
done
echo rc=$?

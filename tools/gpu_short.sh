# Epoch-boundary check: the data-path GPU tests, the boundary probe, the driver-length bench
# (--steps 20 --warmup 5) with its host timeline, and the default-length bench.
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/short.log
: > $L
timeout -k 10 400 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_linear.py tests/test_gpu_app.py tests/test_gpu_cnn_f32.py -x -q --timeout 120 --timeout-method thread >> $L 2>&1 || exit 1
timeout -k 10 120 python tools/boundary_probe.py >> $L 2>&1 || exit 1
for i in 1 2 3; do
  PDM_BENCH_DEBUG=1 timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 >> $L 2>&1 || exit 1
done
PDM_BENCH_DEBUG=1 timeout -k 10 120 python bench.py --gpus 1 --steps 200 --warmup 30 >> $L 2>&1 || exit 1
echo done >> $L

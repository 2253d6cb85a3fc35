# Full GPU test suite, then in-step kernel traces (tools/gpu_trace.sh) at the given batches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
bash tools/gpu_trace.sh "$@"

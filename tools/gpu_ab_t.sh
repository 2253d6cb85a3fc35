# exact backward tests on the in-tree build, then the interleaved A/B against $@
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_cnn_bwd_exact.py tests/test_gpu_cnn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || exit 1
bash tools/gpu_ab.sh "$@"

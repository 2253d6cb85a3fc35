# New GPU tests of this round, then the xgmi fixed-cost diagnostics at N=1 forced:
# persistent-launch width 16 / 32 / 64 and the payload-free protocol (PDM_XG_DIAG=1).
set -o pipefail
mkdir -p gpurun_out/r5xg
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_comm.py tests/test_gpu_bench.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5xg/tests.log 2>&1 || exit 1
PDM_FORCE_COMM=1 PDM_COMM=xgmi bash tools/gpu_ab_b.sh "256 32" build/xgwg16 build/xgwg32 build/xgdiag

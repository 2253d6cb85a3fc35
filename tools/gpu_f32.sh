# fp32 CNN path: GPU tests, then per-step timing (bench.py --dtype fp32 at N=1) + kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_cnn_f32.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_f32.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --dtype fp32 --scaling weak --steps 100 --warmup 10 > gpurun_out/bench_f32.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f32 -o run -- python3 bench.py --dtype fp32 --scaling weak --steps 100 --warmup 10 > gpurun_out/prof_f32.log 2>&1
echo rc=$?

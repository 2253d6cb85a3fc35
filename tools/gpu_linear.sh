# Linear (reference Net): GPU tests, bench + kernel trace on one MI355X.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_app.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_lin_tests.log 2>&1 && \
timeout -k 10 120 python bench.py --model linear > gpurun_out/bench_lin.json 2>gpurun_out/bench_lin.err && \
timeout -k 10 120 python bench.py --model linear --steps 20 --warmup 5 > gpurun_out/bench_lin20.json 2>>gpurun_out/bench_lin.err && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lin -o run -- python3 bench.py --model linear --steps 200 --warmup 30 > gpurun_out/prof_lin.log 2>&1
echo rc=$?

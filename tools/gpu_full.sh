# Full GPU test suite + N=1 benches (CNN default + driver-length, Linear) + CNN kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_20.json 2>gpurun_out/bench_20.err && \
timeout -k 10 120 python bench.py > gpurun_out/bench_def.json 2>gpurun_out/bench_def.err && \
timeout -k 10 120 python bench.py --model linear > gpurun_out/bench_lin.json 2>gpurun_out/bench_lin.err && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 200 --warmup 30 > gpurun_out/prof.log 2>&1
echo rc=$?

# Full GPU test suite + N=1 benches (CNN default, driver length, a whole epoch + boundary,
# fp32, the N>1 chain priced with a 1-rank RCCL communicator, Linear) + kernel trace + PMC.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_20.json 2>gpurun_out/bench_20.err && \
timeout -k 10 120 python bench.py > gpurun_out/bench_def.json 2>gpurun_out/bench_def.err && \
timeout -k 10 120 python bench.py --steps 470 > gpurun_out/bench_470.json 2>gpurun_out/bench_470.err && \
timeout -k 10 200 python bench.py --dtype fp32 > gpurun_out/bench_f32.json 2>gpurun_out/bench_f32.err && \
PDM_FORCE_COMM=1 timeout -k 10 200 python bench.py > gpurun_out/bench_fc.json 2>gpurun_out/bench_fc.err && \
timeout -k 10 120 python bench.py --model linear > gpurun_out/bench_lin.json 2>gpurun_out/bench_lin.err && \
timeout -k 10 300 python -u tools/kbench.py 32 64 128 256 > gpurun_out/kbench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 200 --warmup 30 > gpurun_out/prof.log 2>&1 && \
bash tools/pmc_run.sh && bash tools/pmc_bwd.sh
echo rc=$?

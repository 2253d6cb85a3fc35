# Iteration: CNN GPU tests, W1^T double buffer A/B (kbench B=256/1024 + bench, interleaved),
# Linear bench at two lengths + its kernel trace
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/iter.log
: > $L
timeout -k 10 400 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_cnn_f32.py -x -q --timeout 200 --timeout-method thread >> $L 2>&1 || exit 1
for rep in 1 2; do for v in 0 1; do
  echo "wt2=$v" >> $L
  PDM_FC1_WT2=$v timeout -k 10 200 python tools/kbench.py 256 1024 >> $L 2>&1 || exit 1
  PDM_FC1_WT2=$v timeout -k 10 200 python bench.py --scaling weak >> $L 2>&1 || exit 1
done; done
PDM_EXT_PATH=build/stamps/_C.cpython-310-x86_64-linux-gnu.so timeout -k 10 120 python -u tools/stamps.py 256 >> $L 2>&1 || exit 1
echo linear >> $L
timeout -k 10 200 python bench.py --model linear --steps 200 >> $L 2>&1 || exit 1
timeout -k 10 200 python bench.py --model linear --steps 2000 >> $L 2>&1 || exit 1
timeout -k 10 200 python bench.py --model linear --steps 1 --warmup 300 >> $L 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lin -o run -- python3 bench.py --model linear --steps 200 --warmup 30 > gpurun_out/prof_lin.log 2>&1
echo rc=$?

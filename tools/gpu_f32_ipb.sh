# Iteration: CNN + fp32 GPU tests, fp32 conv-backward images-per-workgroup sweep, W1^T
# double buffer on/off and a forward-only band split at B=256 (kbench + bench)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/f32_ipb.log
: > $L
timeout -k 10 400 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_cnn_f32.py -x -q --timeout 200 --timeout-method thread >> $L 2>&1 || exit 1
for i in 1 2 3; do PDM_F32_IPB=$i timeout -k 10 200 python bench.py --dtype fp32 --scaling weak --steps 100 --warmup 10 >> $L 2>&1 || exit 1; done
for v in 0 1; do echo "wt2=$v" >> $L; PDM_FC1_WT2=$v timeout -k 10 200 python tools/kbench.py 256 >> $L 2>&1 || exit 1; done
for fb in 2 3; do echo "fwd_bands=$fb" >> $L; PDM_FWD_BANDS=$fb timeout -k 10 200 python tools/kbench.py 256 >> $L 2>&1 || exit 1; done
for v in 0 1; do PDM_FC1_WT2=$v timeout -k 10 200 python bench.py --scaling weak >> $L 2>&1 || exit 1; done
echo rc=$?

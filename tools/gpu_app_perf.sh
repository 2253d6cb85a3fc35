# The reference CLI end to end on one MI355X (spawn mode, synthetic MNIST, 3 epochs, --perf):
# reference Net (defaults: Adam, fp32) and the CNN (SGD, bf16).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && rm -rf app_run && mkdir app_run && cd app_run
timeout -k 10 300 python $GRAFT_REPO_ROOT/multi_proc_single_gpu.py --world-size 1 --synthetic --epochs 3 --perf > $GRAFT_REPO_ROOT/gpurun_out/app_linear.log 2>&1 && \
timeout -k 10 300 python $GRAFT_REPO_ROOT/multi_proc_single_gpu.py --world-size 1 --synthetic --epochs 3 --perf --arch cnn --optimizer sgd --lr 0.05 > $GRAFT_REPO_ROOT/gpurun_out/app_cnn.log 2>&1
echo rc=$?

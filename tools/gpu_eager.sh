# PyTorch comparison points on one MI355X (tools/reference_eager.py): the reference's own loop
# (DataLoader), device-resident eager, and the whole step captured in a torch.cuda.graph (fp32
# and bf16 autocast); then the fp32 CNN path's kernel trace.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/eager.jsonl
for v in "--loader dataloader" "--loader device" "--loader graph" "--loader graph --amp bf16"; do
  MASTER_PORT=29541 timeout -k 10 300 python tools/reference_eager.py $v --steps 200 --warmup 30 >> gpurun_out/eager.jsonl 2>gpurun_out/eager.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f32 -o run -- python3 bench.py --dtype fp32 --steps 100 --warmup 10 > gpurun_out/prof_f32.log 2>&1
echo rc=$?

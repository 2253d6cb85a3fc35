# Driver-length bench (--steps 20 --warmup 5) next to the default length, and the small
# per-rank batches (strong-scaling shapes) at N=1: local chain and the N>1 chain priced with a
# 1-rank communicator.
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/short.log
: > $L
for i in 1 2; do
  PDM_BENCH_DEBUG=1 timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 >> $L 2>&1 || exit 1
  PDM_BENCH_DEBUG=1 timeout -k 10 120 python bench.py --gpus 1 --steps 200 --warmup 30 >> $L 2>&1 || exit 1
done
for B in 32 64; do
  PDM_BENCH_DEBUG=1 timeout -k 10 120 python bench.py --scaling weak --batch-per-rank $B >> $L 2>&1 || exit 1
  PDM_FORCE_COMM=1 timeout -k 10 200 python bench.py --scaling weak --batch-per-rank $B >> $L 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/kbench.py 32 64 >> $L 2>&1 || exit 1
echo done >> $L

# Driver-length bench (--steps 20 --warmup 5): epoch boundary variants, interleaved.
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/short.log
: > $L
for i in 1 2; do
  for e in "X=1" "PDM_BENCH_BOUNDARY=0" "PDM_GATHER_AHEAD=0"; do
    echo "== $e" >> $L
    env $e timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 >> $L 2>&1 || exit 1
  done
done
echo "== 200 steps" >> $L
timeout -k 10 120 python bench.py --gpus 1 --steps 200 --warmup 30 >> $L 2>&1 || exit 1
echo "== 470 steps" >> $L
timeout -k 10 120 python bench.py --gpus 1 --steps 470 --warmup 30 >> $L 2>&1 || exit 1
echo done >> $L

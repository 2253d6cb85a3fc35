# The driver's window (boundary inside) with the sampler worker's OpenMP threads limited
# (OMP_NUM_THREADS=1) against the box default, interleaved.  bash tools/gpu_r6_omp.sh NAME
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
for rep in 1 2 3 4; do
  PDM_BENCH_DEBUG=1 timeout -k 10 150 python bench.py --steps 20 --warmup 5 >> $O/a.jsonl 2>> $O/a.err || exit 1
  OMP_NUM_THREADS=1 PDM_BENCH_DEBUG=1 timeout -k 10 150 python bench.py --steps 20 --warmup 5 >> $O/b.jsonl 2>> $O/b.err || exit 1
done
echo "OMP_NUM_THREADS=$OMP_NUM_THREADS nproc=$(nproc)"
grep -h window $O/a.err | sed 's/^/A /'; grep -h window $O/b.err | sed 's/^/B /'
grep -h -o '"ms_per_step": [0-9.]*' $O/a.jsonl | sed 's/^/A /'; grep -h -o '"ms_per_step": [0-9.]*' $O/b.jsonl | sed 's/^/B /'

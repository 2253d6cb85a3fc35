# bench.py's driver window with device events at the host marks (PDM_BENCH_DEBUG=events), with
# and without the boundary, untraced.  bash tools/gpu_r6_window3.sh NAME
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
for rep in 1 2 3; do
  PDM_BENCH_DEBUG=events timeout -k 10 150 python bench.py --steps 20 --warmup 5 >> $O/bench.jsonl 2>> $O/debug.err || exit 1
  PDM_BENCH_DEBUG=events PDM_BENCH_BOUNDARY=0 timeout -k 10 150 python bench.py --steps 20 --warmup 5 >> $O/bench_nb.jsonl 2>> $O/debug_nb.err || exit 1
done
grep -h window $O/debug.err $O/debug_nb.err
grep -h -o '"ms_per_step": [0-9.]*' $O/bench.jsonl $O/bench_nb.jsonl

# The driver's 20-step window, dispatch by dispatch: where the time between the ~52 us steady
# steps goes (the ragged tail step, the epoch boundary, host enqueue gaps).
# bash tools/gpu_r6_window.sh NAME -> gpurun_out/NAME/
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  PDM_BENCH_DEBUG=1 timeout -k 10 150 python bench.py --steps 20 --warmup 5 >> $O/bench.jsonl 2>> $O/bench_debug.err || exit 1
  PDM_BENCH_BOUNDARY=0 timeout -k 10 150 python bench.py --steps 20 --warmup 5 >> $O/bench_noboundary.jsonl 2>> $O/bench.err || exit 1
done
t=$O/tr
timeout -k 10 150 rocprofv3 --kernel-trace -d $t -o run -- python3 bench.py --steps 20 --warmup 5 > $O/tr.log 2>&1 || exit 1
python tools/rocpd_timeline.py $(ls $t/*/*.db $t/*.db 2>/dev/null | head -1) --last 200 --count 200 --title "driver window, B=256" > $O/timeline.md
cp $(ls $t/*/*.db $t/*.db 2>/dev/null | head -1) $O/run.db
rm -rf $t
echo done

# Round-5 baseline on a fresh box: GPU suite, driver-length and 200-step benches, the
# world-size>1 chain at the strong-scaling per-rank batches (PDM_FORCE_COMM=1), BASELINE
# config 5 (large per-rank batch, enlarged synthetic set) with an in-step trace at 8192.
# Everything lands in gpurun_out/r5base/.
set -o pipefail
O=gpurun_out/r5base
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
: > $O/bench.jsonl
run() { echo "## $*" >> $O/bench.jsonl; timeout -k 10 200 "$@" >> $O/bench.jsonl 2>> $O/bench.err || exit 1; }
run python bench.py --gpus 1 --steps 20 --warmup 5
run python bench.py --gpus 1 --steps 20 --warmup 5
run python bench.py
for B in 32 64; do
  PDM_FORCE_COMM=1 run python bench.py --scaling weak --batch-per-rank $B
done
for B in 4096 8192; do
  run python bench.py --scaling weak --batch-per-rank $B --train-size 262144 --steps 40 --warmup 8
done
d=$O/trace_8192
timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --scaling weak --batch-per-rank 8192 --train-size 262144 --steps 40 --warmup 8 > /dev/null 2>&1 || exit 1
python tools/rocpd_summary.py $(ls $d/*.db) --title "in-step kernels, bench.py B=8192 (train set 262144), 40 steps" --steps 30 > $O/trace_8192.md && rm -rf $d
echo done >> $O/bench.jsonl

# Large per-rank batch (BASELINE config 5): fc1_fwd tests incl. the 128-row blocks, the
# graph-replayed 8192 epoch, benches at 4096 / 8192 over an enlarged synthetic set, and an
# in-step trace at 8192.  Output: gpurun_out/r5big/
set -o pipefail
O=gpurun_out/r5big
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_cnn.py -x -q -k "fc1_fwd or large_batch or autograd" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
: > $O/bench.jsonl
for B in 4096 8192; do
  echo "## B=$B" >> $O/bench.jsonl
  timeout -k 10 200 python bench.py --scaling weak --batch-per-rank $B --train-size 262144 --steps 40 --warmup 8 >> $O/bench.jsonl 2>> $O/bench.err || exit 1
done
d=$O/trace_8192
timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --scaling weak --batch-per-rank 8192 --train-size 262144 --steps 40 --warmup 8 > /dev/null 2>&1 || exit 1
python tools/rocpd_summary.py $(ls $d/*.db) --title "in-step kernels, bench.py B=8192 (train set 262144), 40 steps" --steps 30 > $O/trace_8192.md && rm -rf $d

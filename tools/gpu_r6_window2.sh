# The driver's 20-step window with the HIP runtime and memory-copy domains traced (no PMC):
# what the host enqueues at the epoch boundary and at each graph replay.
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
t=$O/tr
PDM_BENCH_DEBUG=1 timeout -k 10 150 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d $t -o run -- python3 bench.py --steps 20 --warmup 5 > $O/tr.log 2>&1 || exit 1
cp $(ls $t/*/*.db $t/*.db 2>/dev/null | head -1) $O/run.db
rm -rf $t
echo done

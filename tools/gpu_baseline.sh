# Start-of-round check: full GPU suite + driver-length and default benches.
set -o pipefail
O=gpurun_out/base
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
: > $O/bench.jsonl
run() { timeout -k 10 240 "$@" >> $O/bench.jsonl 2>> $O/bench.err || exit 1; }
run python bench.py --gpus 1 --steps 20 --warmup 5
run python bench.py --gpus 1 --steps 20 --warmup 5
run python bench.py
echo done

# Final check of the tree as committed: the full GPU suite, __graft_entry__.smoke(), the
# driver-length bench and the fp32 bench (gpurun_out/final/)
set -o pipefail
O=gpurun_out/final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || exit 1
: > $O/bench.jsonl
for a in "--gpus 1 --steps 20 --warmup 5" "" "--dtype fp32"; do
  echo "## python bench.py $a" >> $O/bench.jsonl
  timeout -k 10 150 python bench.py $a >> $O/bench.jsonl 2>> $O/bench.err || exit 1
done
echo done

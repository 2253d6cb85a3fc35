# fp32 split-bf16 iteration: tests, bench, in-step trace
set -o pipefail
O=gpurun_out/r4c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cnn_f32.py tests/test_gpu_app.py -v --timeout 300 --timeout-method thread > $O/f32_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
: > $O/bench.jsonl
for rep in 1 2; do
  timeout -k 10 240 python bench.py --dtype fp32 --scaling weak >> $O/bench.jsonl 2>> $O/bench.err || exit 1
done
d=$O/trace_f32x3
timeout -k 10 180 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --dtype fp32 --steps 200 --warmup 30 --scaling weak > /dev/null 2>&1 || exit 1
python tools/rocpd_summary.py $(ls $d/*.db) --title "in-step kernels, bench.py --dtype fp32 (split-bf16) B=256, 200 steps" --steps 150 > $O/trace_f32x3.md && rm -rf $d
echo done

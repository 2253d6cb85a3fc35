# fp32 split-bf16 conv backward v2 (next image prefetched under compute, batched scatter
# loads): correctness with the variant build, then interleaved A/B and a trace
set -o pipefail
O=gpurun_out/r4e
mkdir -p $O
export TMPDIR=/tmp
V=build/x3v2/_C.cpython-310-x86_64-linux-gnu.so
PDM_EXT_PATH=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_cnn_f32.py -x -v --timeout 200 --timeout-method thread > $O/f32_tests_v2.log 2>&1 || exit 1
: > $O/ab.jsonl
for rep in 1 2; do
  for v in "" $V; do
    echo "rep=$rep ext=${v:-tree}" >> $O/ab.jsonl
    PDM_EXT_PATH=$v timeout -k 10 240 python bench.py --dtype fp32 --steps 100 --warmup 20 --scaling weak >> $O/ab.jsonl 2>> $O/bench.err || exit 1
  done
done
d=$O/tr_v2
PDM_EXT_PATH=$V timeout -k 10 180 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --dtype fp32 --steps 100 --warmup 20 --scaling weak > /dev/null 2>&1 || exit 1
python tools/rocpd_summary.py $(ls $d/*.db) --title "x3v2" --steps 80 > $O/trace_v2.md && rm -rf $d
echo done

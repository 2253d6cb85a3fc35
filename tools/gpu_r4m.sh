# fp32 split-bf16 conv backward: whole-window dz2 scatter (no per-unit zeroing).
# conv backward issues its first unit's loads ahead of the W2^T copy.  fp32 tests, phase
# stamps, interleaved A/B against the refresh tree (build/wt_head: its own Python and .so).
set -o pipefail
O=gpurun_out/r4m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cnn_f32.py tests/test_gpu_app.py -k "f32 or fp32" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
PDM_EXT_PATH=build/stamps_f32/_C.cpython-310-x86_64-linux-gnu.so timeout -k 10 120 python tools/stamps_f32.py 256 > $O/stamps_256.txt 2>&1 || exit 1
: > $O/ab.jsonl
R=$PWD
for rep in 1 2; do
  for v in wt_head tree; do
    echo "## rep=$rep $v" >> $O/ab.jsonl
    if [ $v = tree ]; then d=$R; else d=$R/build/$v; fi
    ( cd $d && timeout -k 10 150 python bench.py --dtype fp32 --steps 200 --warmup 30 --scaling weak ) >> $O/ab.jsonl 2>> $O/bench.err || exit 1
    if [ $rep = 1 ]; then
      t=$R/$O/tr_$v
      ( cd $d && timeout -k 10 150 rocprofv3 --kernel-trace -d $t -o run -- python3 bench.py --dtype fp32 --steps 100 --warmup 20 --scaling weak > /dev/null 2>&1 ) || exit 1
      python tools/rocpd_summary.py $(ls $t/*.db) --title "fp32 $v" --steps 80 > $O/trace_$v.md; rm -rf $t
    fi
  done
done
echo done

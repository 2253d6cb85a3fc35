# fp32 forward: split pinned ahead of conv1 (pin) and tap-pipelined conv2 (tree) vs HEAD (base);
# fc1_fwd split-K 96 at the strong-scaling batches (PDM_SPLITK_CAP=96 vs 32), local and
# world-size>1 chains.  Interleaved, twice; in-step traces summarised on the box.
set -o pipefail
O=gpurun_out/r4g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cnn_f32.py tests/test_gpu_cnn.py -k "f32 or split_k or forward" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
: > $O/f32.jsonl
for rep in 1 2; do
  for v in build/base build/pin ""; do
    tag=$(echo "${v:-tree}" | tr '/' '_')
    if [ -n "$v" ]; then export PDM_EXT_PATH=$v/_C.cpython-310-x86_64-linux-gnu.so; else unset PDM_EXT_PATH; fi
    echo "rep=$rep $tag" >> $O/f32.jsonl
    timeout -k 10 240 python bench.py --dtype fp32 --steps 100 --warmup 20 --scaling weak >> $O/f32.jsonl 2>> $O/bench.err || exit 1
    if [ $rep = 1 ]; then
      d=$O/tr_$tag
      timeout -k 10 180 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --dtype fp32 --steps 60 --warmup 10 --scaling weak > /dev/null 2>&1 || exit 1
      python tools/rocpd_summary.py $(ls $d/*.db) --title "fp32 $tag" --steps 50 > $O/trace_f32_$tag.md; rm -rf $d
    fi
  done
done
unset PDM_EXT_PATH
: > $O/splitk.jsonl
for rep in 1 2; do
  for cap in 32 96; do
    for B in 32 64; do
      for f in 0 1; do
        echo "rep=$rep cap=$cap B=$B force=$f" >> $O/splitk.jsonl
        PDM_SPLITK_CAP=$cap PDM_FORCE_COMM=$f timeout -k 10 120 python bench.py --scaling weak --batch-per-rank $B >> $O/splitk.jsonl 2>> $O/bench.err || exit 1
      done
      if [ $rep = 1 ]; then
        d=$O/tr_cap${cap}_$B
        PDM_SPLITK_CAP=$cap PDM_FORCE_COMM=1 timeout -k 10 180 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --scaling weak --batch-per-rank $B --steps 200 --warmup 30 > /dev/null 2>&1 || exit 1
        python tools/rocpd_summary.py $(ls $d/*.db) --title "force-comm B=$B splitk cap $cap" --steps 150 > $O/trace_cap${cap}_$B.md; rm -rf $d
      fi
    done
  done
done
echo done

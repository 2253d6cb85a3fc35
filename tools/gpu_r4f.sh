# fp32 split-bf16: forward phase ablations (timing only) + conv-backward images per workgroup
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cnn_f32.py tests/test_gpu_app.py -x -v --timeout 300 --timeout-method thread > $O/f32_tests.log 2>&1 || exit 1
for v in "" build/abl21 build/abl22 build/abl23; do
  tag=$(echo "${v:-tree}" | tr '/' '_')
  if [ -n "$v" ]; then export PDM_EXT_PATH=$v/_C.cpython-310-x86_64-linux-gnu.so; else unset PDM_EXT_PATH; fi
  d=$O/tr_$tag
  timeout -k 10 180 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --dtype fp32 --steps 60 --warmup 10 --scaling weak > $O/$tag.json 2>&1
  python tools/rocpd_summary.py $(ls $d/*.db) --title "$tag" --steps 50 > $O/trace_$tag.md; rm -rf $d
done
unset PDM_EXT_PATH
: > $O/ipb.jsonl
for rep in 1 2; do
  for ipb in 3 5 7; do
    echo "rep=$rep ipb=$ipb" >> $O/ipb.jsonl
    PDM_F32_IPB=$ipb timeout -k 10 240 python bench.py --dtype fp32 --steps 100 --warmup 20 --scaling weak >> $O/ipb.jsonl 2>> $O/bench.err || exit 1
  done
done
echo done

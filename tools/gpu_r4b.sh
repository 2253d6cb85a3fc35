# Round 4: fp32 split-bf16 tuning A/B (conv-backward images per workgroup, balanced dgrad
# build), each bench run twice interleaved.
set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
export TMPDIR=/tmp
: > $O/f32ab.jsonl
for rep in 1 2; do
  for v in "" build/x3bal; do
    if [ -n "$v" ]; then export PDM_EXT_PATH=$v/_C.cpython-310-x86_64-linux-gnu.so; else unset PDM_EXT_PATH; fi
    for ipb in 1 2 3 7; do
      echo "rep=$rep ext=${v:-tree} ipb=$ipb" >> $O/f32ab.jsonl
      PDM_F32_IPB=$ipb timeout -k 10 240 python bench.py --dtype fp32 --steps 100 --warmup 20 --scaling weak >> $O/f32ab.jsonl 2>> $O/bench.err || exit 1
    done
  done
done
unset PDM_EXT_PATH
d=$O/trace_f32x3
timeout -k 10 180 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --dtype fp32 --steps 200 --warmup 30 --scaling weak > /dev/null 2>&1 || exit 1
python tools/rocpd_summary.py $(ls $d/*.db) --title "in-step kernels, bench.py --dtype fp32 (split-bf16 conv2) B=256, 200 steps" --steps 150 > $O/trace_f32x3.md && rm -rf $d
echo done

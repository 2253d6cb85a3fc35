# fp32 split-bf16 conv backward: phase ablations (timing only) via in-step kernel traces
set -o pipefail
O=gpurun_out/r4d
mkdir -p $O
export TMPDIR=/tmp
for v in "" build/abl11 build/abl12 build/abl13; do
  tag=$(echo "${v:-tree}" | tr '/' '_')
  if [ -n "$v" ]; then export PDM_EXT_PATH=$v/_C.cpython-310-x86_64-linux-gnu.so; else unset PDM_EXT_PATH; fi
  d=$O/tr_$tag
  timeout -k 10 180 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --dtype fp32 --steps 100 --warmup 20 --scaling weak > $O/$tag.json 2>&1 || exit 1
  python tools/rocpd_summary.py $(ls $d/*.db) --title "$tag" --steps 80 > $O/trace_$tag.md && rm -rf $d
done
echo done

# bash tools/gpu_ab_b.sh "32 256" build/a ... : interleaved A/B of extension builds at the given
# per-rank batches -- bench.py (local chain, 200 steps) and an in-step rocprofv3 kernel trace
# per batch and variant, twice (the in-tree build is the first variant).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/abb.log
export TMPDIR=/tmp
BS="$1"; shift
for rep in 1 2; do
for v in "" "$@"; do
  tag=$(echo "${v:-default}" | tr '/' '_')
  if [ -n "$v" ]; then export PDM_EXT_PATH=$v/_C.cpython-310-x86_64-linux-gnu.so; else unset PDM_EXT_PATH; fi
  for B in $BS; do
    echo "== rep $rep variant ${v:-default} B=$B" >> gpurun_out/abb.log
    timeout -k 10 120 python bench.py --scaling weak --batch-per-rank $B >> gpurun_out/abb.log 2>&1 || exit 1
    d=gpurun_out/abb_prof/${rep}_${tag}_$B
    timeout -k 10 180 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --scaling weak --batch-per-rank $B --steps 200 --warmup 30 > /dev/null 2>&1 || exit 1
    python tools/rocpd_summary.py $(ls $d/*.db | head -1) --title "rep $rep ${v:-default} B=$B" --steps 150 > ${d}.md && rm -rf $d
  done
done
done
echo rc=$?

# BS="32 256" bash tools/gpu_env_ab.sh "VAR=a" "VAR=b" ... : interleaved A/B of environment
# settings (the first variant is the defaults): per per-rank batch (BS, default 256) bench.py
# (local chain, 200 steps) and an in-step rocprofv3 kernel trace, summarised on the box
# (tools/rocpd_summary.py), twice.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/env_ab.log
export TMPDIR=/tmp
for rep in 1 2; do
for e in "" "$@"; do
  tag=$(echo "${e:-default}" | tr '/=' '__')
  for B in ${BS:-256}; do
    echo "== rep $rep env ${e:-default} B=$B" >> gpurun_out/env_ab.log
    d=gpurun_out/env_prof/${rep}_${tag}_$B
    ( if [ -n "$e" ]; then export "$e"; fi
      timeout -k 10 120 python bench.py --scaling weak --batch-per-rank $B >> gpurun_out/env_ab.log 2>&1 && \
      timeout -k 10 180 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --scaling weak --batch-per-rank $B --steps 200 --warmup 30 > /dev/null 2>&1 ) || exit 1
    python tools/rocpd_summary.py $(ls $d/*.db | head -1) --title "rep $rep ${e:-default} B=$B" --steps 150 > ${d}.md && rm -rf $d
  done
done
done
echo rc=$?

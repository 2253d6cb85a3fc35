# bash tools/gpu_env_ab.sh "VAR=a" "VAR=b" ... : interleaved bench + in-step kernel trace per
# environment setting (the first argument "" = defaults), twice
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/env_ab.log
export TMPDIR=/tmp
for rep in 1 2; do
for e in "" "$@"; do
  tag=$(echo "${e:-default}" | tr '/=' '__')
  echo "== rep $rep env ${e:-default}" >> gpurun_out/env_ab.log
  ( if [ -n "$e" ]; then export "$e"; fi
    timeout -k 10 120 python bench.py >> gpurun_out/env_ab.log 2>&1 && \
    timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/env_prof/${rep}_$tag -o run -- python3 bench.py --steps 200 --warmup 30 > /dev/null 2>&1 ) || exit 1
done
done
echo rc=$?

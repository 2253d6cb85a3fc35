# bash tools/gpu_ab.sh build/a build/b ... : interleaved kbench (256, 1024) + bench + in-step
# kernel trace per variant, twice (default = the in-tree build)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab.log
export TMPDIR=/tmp
for rep in 1 2; do
for v in "" "$@"; do
  tag=$(echo "${v:-default}" | tr '/' '_')
  echo "== rep $rep variant ${v:-default}" >> gpurun_out/ab.log
  if [ -n "$v" ]; then export PDM_EXT_PATH=$v/_C.cpython-310-x86_64-linux-gnu.so; else unset PDM_EXT_PATH; fi
  timeout -k 10 200 python -u tools/kbench.py 256 1024 >> gpurun_out/ab.log 2>&1 || exit 1
  timeout -k 10 120 python bench.py >> gpurun_out/ab.log 2>&1 || exit 1
  timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/ab_prof/${rep}_$tag -o run -- python3 bench.py --steps 200 --warmup 30 > /dev/null 2>&1 || exit 1
done
done
echo rc=$?

# bash tools/gpu_variants.sh build/a build/b ... : bwd-exact test + kbench 256/1024 per variant
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/variants.log
for v in "" "$@"; do
  echo "== variant ${v:-default}" >> gpurun_out/variants.log
  if [ -n "$v" ]; then export PDM_EXT_PATH=$v/_C.cpython-310-x86_64-linux-gnu.so; fi
  timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cnn_bwd_exact.py >> gpurun_out/variants.log 2>&1 || exit 1
  timeout -k 10 200 python -u tools/kbench.py 256 1024 >> gpurun_out/variants.log 2>&1 || exit 1
done
echo rc=$?

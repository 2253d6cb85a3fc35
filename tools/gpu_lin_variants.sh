# bash tools/gpu_lin_variants.sh build/a ... : linear tests + linear bench per variant, CNN bench (default)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/lin_variants.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_optim.py -x -q --timeout 120 --timeout-method thread >> gpurun_out/lin_variants.log 2>&1 || exit 1
timeout -k 10 120 python bench.py >> gpurun_out/lin_variants.log 2>&1 || exit 1
for v in "" "$@"; do
  echo "== variant ${v:-default}" >> gpurun_out/lin_variants.log
  if [ -n "$v" ]; then export PDM_EXT_PATH=$v/_C.cpython-310-x86_64-linux-gnu.so; fi
  timeout -k 10 120 python bench.py --model linear >> gpurun_out/lin_variants.log 2>&1 || exit 1
  timeout -k 10 120 python bench.py --model linear --optimizer sgd >> gpurun_out/lin_variants.log 2>&1 || exit 1
done
echo rc=$?

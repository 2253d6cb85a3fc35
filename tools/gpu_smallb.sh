# Small-batch pricing: comm/bench GPU tests, per-kernel times at B = 32..256 and the
# full N>1 step chain at N = 1 (PDM_FORCE_COMM=1: 1-rank communicator) per transport
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_bench.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_comm.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/kbench.py 32 64 128 256 > gpurun_out/kb_base.log 2>&1 || exit 1
: > gpurun_out/fc_base.log
for B in 32 64 128 256; do
  for T in rccl xgmi; do
    PDM_FORCE_COMM=1 PDM_COMM=$T timeout -k 10 120 python bench.py --scaling weak --batch-per-rank $B --steps 200 --warmup 30 >> gpurun_out/fc_base.log 2>&1 || exit 1
  done
  timeout -k 10 120 python bench.py --scaling weak --batch-per-rank $B --steps 200 --warmup 30 >> gpurun_out/fc_base.log 2>&1 || exit 1
done
echo rc=$?

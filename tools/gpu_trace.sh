# In-step kernel traces of bench.py at the given per-rank batches (N=1: the local chain and
# the world-size>1 chain through a 1-rank RCCL communicator).  Usage: bash tools/gpu_trace.sh 32 64
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in "$@"; do
  timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/tr/local_$B -o run -- python3 bench.py --scaling weak --batch-per-rank $B --steps 200 --warmup 30 > gpurun_out/tr_local_$B.log 2>&1 || exit 1
  PDM_FORCE_COMM=1 PDM_COMM=rccl timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/tr/rccl_$B -o run -- python3 bench.py --scaling weak --batch-per-rank $B --steps 200 --warmup 30 > gpurun_out/tr_rccl_$B.log 2>&1 || exit 1
done
echo rc=$?

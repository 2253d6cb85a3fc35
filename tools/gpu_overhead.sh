set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/overhead.log
for k in 4 8 20 100 400; do
  timeout -k 10 180 python -u bench.py --steps $k --warmup 5 >> gpurun_out/overhead.log 2>>gpurun_out/overhead.err || exit 1
done
echo done

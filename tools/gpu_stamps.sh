set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/stamps256.log
for v in build/stamps ${EXTRA_VARIANTS}; do
  echo "== $v" >> gpurun_out/stamps256.log
  PDM_EXT_PATH=$v/_C.cpython-310-x86_64-linux-gnu.so timeout -k 10 120 python -u tools/stamps.py ${1:-256} >> gpurun_out/stamps256.log 2>&1 || exit 1
done
echo rc=$?

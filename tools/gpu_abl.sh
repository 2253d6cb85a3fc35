set -o pipefail
mkdir -p gpurun_out
for v in 1 2 3; do
  PDM_EXT_PATH=build/abl$v/_C.cpython-310-x86_64-linux-gnu.so timeout -k 10 120 python -u tools/stamps.py 256 > gpurun_out/abl$v.log 2>&1 || exit 1
done
PDM_EXT_PATH=build/m6/_C.cpython-310-x86_64-linux-gnu.so timeout -k 10 200 python -u tools/kbench.py 256 1024 > gpurun_out/kb_m6.log 2>&1
echo rc=$?

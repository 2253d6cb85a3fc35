set -o pipefail
O=gpurun_out/r4l
mkdir -p $O
export TMPDIR=/tmp
PDM_EXT_PATH=build/stamps_f32/_C.cpython-310-x86_64-linux-gnu.so timeout -k 10 120 python tools/stamps_f32.py 256 > $O/stamps_256.txt 2>&1 || exit 1
timeout -k 10 150 python bench.py --dtype fp32 --steps 200 --warmup 30 > $O/bench.json 2>&1 || exit 1
echo done

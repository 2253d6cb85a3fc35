# fp32 split-bf16 phase stamps (f32x3_fwd / f32x3_conv_bwd) + the fp32 tests of the tree
set -o pipefail
O=gpurun_out/r4h
mkdir -p $O
export TMPDIR=/tmp
PDM_EXT_PATH=build/stamps_f32/_C.cpython-310-x86_64-linux-gnu.so timeout -k 10 300 python tools/stamps_f32.py 256 > $O/stamps_256.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_cnn_f32.py tests/test_gpu_app.py -k "f32 or fp32" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo done

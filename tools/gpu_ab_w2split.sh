set -o pipefail
O=gpurun_out/r4n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cnn_f32.py tests/test_gpu_app.py tests/test_gpu_optim.py -k "f32 or fp32 or optim" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
PDM_EXT_PATH=build/stamps_f32/_C.cpython-310-x86_64-linux-gnu.so timeout -k 10 120 python tools/stamps_f32.py 256 > $O/stamps_256.txt 2>&1 || exit 1
bash tools/gpu_ab_tree.sh r4n_ab "--dtype fp32 --steps 200 --warmup 30 --scaling weak" build/wt_head || exit 1
echo done

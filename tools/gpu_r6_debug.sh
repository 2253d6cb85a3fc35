# bash tools/gpu_r6_debug.sh NAME [pytest args...]: the GPU test suite against the debug-bounds
# build (PDM_DEBUG_BOUNDS=1 python -m pytorch_distributed_mnist_amd.build --out
# build/debug/_C.cpython-310-x86_64-linux-gnu.so), with device printf visible (-s); every
# subprocess the tests start (bench.py, the CLI) loads the same build through PDM_EXT_PATH.
# The log is then searched for failed checks.  -> gpurun_out/NAME/
set -o pipefail
name=$1; shift
O=gpurun_out/$name
mkdir -p $O
export TMPDIR=/tmp
export PDM_EXT_PATH=$PWD/build/debug/_C.cpython-310-x86_64-linux-gnu.so
timeout -k 10 1050 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu "${@:-tests}" > $O/gpu_tests_debug.log 2>&1
rc=$?
tail -5 $O/gpu_tests_debug.log
n=$(grep -c "PDM_CHECK failed" $O/gpu_tests_debug.log || true)
echo "PDM_CHECK failures: $n" | tee $O/check_failures.txt
grep "PDM_CHECK failed" $O/gpu_tests_debug.log | sort | uniq -c | head -50 >> $O/check_failures.txt
exit $rc

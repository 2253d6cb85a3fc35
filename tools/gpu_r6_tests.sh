# bash tools/gpu_r6_tests.sh NAME [pytest args...]: the GPU test suite (or the given tests) of
# the in-tree build, one pytest process, then smoke().  -> gpurun_out/NAME/
set -o pipefail
name=$1; shift
O=gpurun_out/$name
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "${@:-tests}" > $O/gpu_tests.log 2>&1
rc=$?
tail -5 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log

# bash tools/gpu_r6_ab.sh NAME BASE_SO [TESTS...]: GPU tests of the in-tree build (optional),
# then an interleaved A/B of the in-tree extension against BASE_SO (PDM_EXT_PATH): bench.py
# at the driver's window and 200 steps (B = 256) and B = 32, twice; one in-step kernel trace
# per variant; a PMC table per variant at B = 256.  -> gpurun_out/NAME/
set -o pipefail
name=$1; base=$2; shift 2
O=gpurun_out/$name
mkdir -p $O
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$@" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
fi
: > $O/ab.jsonl
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export PDM_EXT_PATH=$base; else unset PDM_EXT_PATH; fi
    for args in "--steps 20 --warmup 5" "" "--scaling weak --batch-per-rank 32"; do
      echo "## rep=$rep $v $args" >> $O/ab.jsonl
      timeout -k 10 150 python bench.py $args >> $O/ab.jsonl 2>> $O/bench.err || exit 1
    done
    if [ $rep = 1 ]; then
      t=$O/tr_$v
      timeout -k 10 150 rocprofv3 --kernel-trace -d $t -o run -- python3 bench.py --steps 200 --warmup 30 > /dev/null 2>&1 || exit 1
      python tools/rocpd_summary.py $(ls $t/*.db) --title "$v: bench.py B=256" --steps 150 > $O/trace_$v.md; rm -rf $t
      t=$O/tr32_$v
      timeout -k 10 150 rocprofv3 --kernel-trace -d $t -o run -- python3 bench.py --scaling weak --batch-per-rank 32 --steps 200 --warmup 30 > /dev/null 2>&1 || exit 1
      python tools/rocpd_summary.py $(ls $t/*.db) --title "$v: bench.py B=32" --steps 150 > $O/trace32_$v.md; rm -rf $t
    fi
  done
done
python tools/refresh_summary.py $O/ab.jsonl > $O/ab_table.md 2>/dev/null
for v in base new; do
  if [ $v = base ]; then export PDM_EXT_PATH=$base; else unset PDM_EXT_PATH; fi
  bash tools/pmc_run.sh ${name}_$v 256 bf16 > $O/pmc_$v.log 2>&1 || exit 1
  cp gpurun_out/pmc/${name}_$v.md $O/pmc_$v.md && rm -rf gpurun_out/pmc/${name}_$v
done
echo done

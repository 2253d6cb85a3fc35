# Round-end refresh of the measured state: full GPU test suite, N=1 benches (driver length,
# default, fp32 split-bf16 / exact, the N>1 chain priced through a 1-rank RCCL communicator,
# Linear, the strong-scaling per-rank batches, the self-spawned two-rank rehearsal), kbench,
# in-step kernel traces summarised on the box, PMC tables, fp32 phase stamps.  Ordered by
# importance (a late step that runs out of time loses the least).  Everything lands in
# gpurun_out/refresh/ (small text files).
set -o pipefail
O=gpurun_out/refresh
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
: > $O/bench.jsonl
run() { echo "## $*" >> $O/bench.jsonl; timeout -k 10 150 "$@" >> $O/bench.jsonl 2>> $O/bench.err || exit 1; }
run python bench.py --gpus 1 --steps 20 --warmup 5
run python bench.py --gpus 1 --steps 20 --warmup 5
run python bench.py
run python bench.py --dtype fp32
PDM_F32_CONV=exact run python bench.py --dtype fp32
PDM_FORCE_COMM=1 run python bench.py
run python bench.py --model linear
for B in 32 64; do
  run python bench.py --scaling weak --batch-per-rank $B
  PDM_FORCE_COMM=1 run python bench.py --scaling weak --batch-per-rank $B
done
PDM_SHARE_DEVICE=1 PDM_BENCH_BACKEND=gloo run python bench.py --gpus 2 --steps 20 --warmup 5
for B in 256 32; do
  d=$O/trace_$B
  timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --scaling weak --batch-per-rank $B --steps 200 --warmup 30 > /dev/null 2>&1 || exit 1
  python tools/rocpd_summary.py $(ls $d/*.db) --title "in-step kernels, bench.py B=$B, 200 steps" --steps 150 > $O/trace_$B.md && rm -rf $d
done
d=$O/trace_f32
timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --dtype fp32 --steps 200 --warmup 30 > /dev/null 2>&1 || exit 1
python tools/rocpd_summary.py $(ls $d/*.db) --title "in-step kernels, bench.py --dtype fp32 (split-bf16) B=256, 200 steps" --steps 150 > $O/trace_f32.md && rm -rf $d
PDM_EXT_PATH=build/stamps_f32/_C.cpython-310-x86_64-linux-gnu.so timeout -k 10 120 python tools/stamps_f32.py 256 > $O/stamps_f32.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/kbench.py 32 64 256 1024 > $O/kbench.log 2>&1 || exit 1
bash tools/pmc_run.sh b256 256 bf16 > $O/pmc_b256.log 2>&1 || exit 1
bash tools/pmc_run.sh f32 256 fp32 > $O/pmc_f32.log 2>&1 || exit 1
bash tools/pmc_run.sh b32force 32 bf16 force > $O/pmc_b32.log 2>&1 || exit 1
cp gpurun_out/pmc/*.md $O/ && rm -rf gpurun_out/pmc
echo rc=$?
# (round-4 final refresh; copy of tools/gpu_refresh.sh)

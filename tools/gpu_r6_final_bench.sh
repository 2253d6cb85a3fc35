# Round-6 end refresh (bash tools/gpu_r6_final_bench.sh [NAME]): every bench configuration, in-step traces, kbench, PMC (B=256).
# Output: gpurun_out/NAME/ (bench.jsonl: one "## command" line, then its JSON line).
set -o pipefail
O=gpurun_out/${1:-r6final}
mkdir -p $O
export TMPDIR=/tmp
: > $O/bench.jsonl
run() { echo "## $*" >> $O/bench.jsonl; timeout -k 10 200 "$@" >> $O/bench.jsonl 2>> $O/bench.err || exit 1; }
run python bench.py --gpus 1 --steps 20 --warmup 5
run python bench.py --gpus 1 --steps 20 --warmup 5
run python bench.py
run python bench.py --gpus 1 --steps 20 --warmup 5
run python bench.py
run python bench.py --dtype fp32
PDM_F32_CONV=exact run python bench.py --dtype fp32
run python bench.py --model linear
PDM_FORCE_COMM=1 run python bench.py --scaling weak
for B in 32 64; do
  run python bench.py --scaling weak --batch-per-rank $B
  PDM_FORCE_COMM=1 run python bench.py --scaling weak --batch-per-rank $B
done
PDM_FORCE_COMM=1 PDM_EMULATE_WS=8 PDM_RCCL_MODE=zero PDM_COMM=rccl run python bench.py --scaling weak --batch-per-rank 32
PDM_FORCE_COMM=1 PDM_EMULATE_WS=4 PDM_RCCL_MODE=zero PDM_COMM=rccl run python bench.py --scaling weak --batch-per-rank 64
PDM_FORCE_COMM=1 PDM_EMULATE_WS=8 PDM_RCCL_MODE=zero PDM_COMM=rccl run python bench.py --scaling weak --batch-per-rank 256
for B in 4096 8192; do
  run python bench.py --scaling weak --batch-per-rank $B --train-size 262144 --steps 40 --warmup 8
done
PDM_SHARE_DEVICE=1 PDM_BENCH_BACKEND=gloo run python bench.py --gpus 2 --steps 20 --warmup 5
tr() {   # name args...
  local name=$1; shift
  local d=$O/tr_$name
  timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py "$@" > /dev/null 2>> $O/bench.err || exit 1
  python tools/rocpd_summary.py $(ls $d/*.db) --title "in-step kernels, bench.py $*" --steps 150 > $O/trace_$name.md || exit 1
  rm -rf $d
}
tr 256 --scaling weak --steps 200 --warmup 30
tr 32 --scaling weak --batch-per-rank 32 --steps 200 --warmup 30
PDM_FORCE_COMM=1 tr force_32 --scaling weak --batch-per-rank 32 --steps 200 --warmup 30
tr f32 --dtype fp32 --steps 200 --warmup 30
timeout -k 10 200 python -u tools/kbench.py 32 64 256 1024 > $O/kbench.log 2>&1 || exit 1
bash tools/pmc_run.sh b256 256 bf16 > $O/pmc_b256.log 2>&1 || exit 1
cp gpurun_out/pmc/b256.md $O/ && rm -rf gpurun_out/pmc
python tools/refresh_summary.py $O/bench.jsonl > $O/bench_table.md 2>/dev/null
echo done >> $O/bench.jsonl

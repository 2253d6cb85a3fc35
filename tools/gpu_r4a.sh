# Round 4 probe: new GPU tests, warm-up ramp of the driver's 20-step window, PMC tables
# (B=256 bf16, B=32 bf16 through the N>1 chain, fp32 B=256), an in-step trace of the fp32
# bench and the rccl-early overlap trace at B=32.
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_shard.py tests/test_gpu_comm.py tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread > $O/new_tests.log 2>&1 || exit 1
: > $O/warm.jsonl
for W in 5 50 500 5; do
  timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup $W >> $O/warm.jsonl 2>> $O/bench.err || exit 1
done
timeout -k 10 240 env PDM_F32_CONV=exact python bench.py --dtype fp32 >> $O/warm.jsonl 2>> $O/bench.err || exit 1
timeout -k 10 240 env PDM_F32_CONV=x3 python bench.py --dtype fp32 >> $O/warm.jsonl 2>> $O/bench.err || exit 1
bash tools/pmc_run.sh b256 256 bf16 > $O/pmc_b256.log 2>&1 || exit 1
bash tools/pmc_run.sh b32force 32 bf16 force > $O/pmc_b32.log 2>&1 || exit 1
PDM_F32_CONV=exact bash tools/pmc_run.sh f32 256 fp32 > $O/pmc_f32.log 2>&1 || exit 1
PDM_F32_CONV=x3 bash tools/pmc_run.sh f32x3 256 fp32 > $O/pmc_f32x3.log 2>&1 || exit 1
cp gpurun_out/pmc/*.md $O/
d=$O/trace_f32
PDM_F32_CONV=exact timeout -k 10 180 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --dtype fp32 --steps 200 --warmup 30 > /dev/null 2>&1 || exit 1
python tools/rocpd_summary.py $(ls $d/*.db) --title "in-step kernels, bench.py --dtype fp32 (exact fp32 MFMA) B=256, 200 steps" --steps 150 > $O/trace_f32.md && rm -rf $d
d=$O/trace_f32x3
PDM_F32_CONV=x3 timeout -k 10 180 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --dtype fp32 --steps 200 --warmup 30 > /dev/null 2>&1 || exit 1
python tools/rocpd_summary.py $(ls $d/*.db) --title "in-step kernels, bench.py --dtype fp32 (split-bf16 conv2) B=256, 200 steps" --steps 150 > $O/trace_f32x3.md && rm -rf $d
d=$O/trace_early32
PDM_FORCE_COMM=1 PDM_COMM=rccl PDM_RCCL_MODE=early timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 bench.py --scaling weak --batch-per-rank 32 --steps 200 --warmup 30 > $O/early32.json 2>&1 || exit 1
python tools/overlap.py $d --a 'nccl|rccl|Nccl|Rccl' --b cnn_bwd > $O/overlap_early32.txt 2>&1
python tools/pmc_table.py --trace $d $d > /dev/null 2>&1
rm -rf gpurun_out/pmc $d/*.csv.gz
echo done

# Where the xgmi transport's fixed cost goes at N = 1 (PDM_FORCE_COMM=1: the world-size>1
# chain with a 1-rank transport, no bytes on a link): bench + in-step kernel trace + a
# timeline stretch of each structure, one transport per run (no calibration), at B = 256, 32.
# Output: gpurun_out/xgmi_cost/{bench.jsonl, trace_<name>_<B>.md, timeline_<name>_<B>.md}
set -o pipefail
O=gpurun_out/xgmi_cost
mkdir -p $O
export TMPDIR=/tmp
: > $O/bench.jsonl
one() {   # name B env...
  local name=$1 B=$2; shift 2
  echo "## $name B=$B $*" >> $O/bench.jsonl
  env PDM_FORCE_COMM=1 "$@" timeout -k 10 150 python bench.py --scaling weak --batch-per-rank $B >> $O/bench.jsonl 2>> $O/bench.err || return 1
  local d=$O/tr_${name}_$B
  env PDM_FORCE_COMM=1 "$@" timeout -k 10 150 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --scaling weak --batch-per-rank $B --steps 200 --warmup 30 > /dev/null 2>> $O/bench.err || return 1
  python tools/rocpd_summary.py $(ls $d/*.db) --title "in-step kernels, $name B=$B (PDM_FORCE_COMM=1 $*)" --steps 150 > $O/trace_${name}_$B.md || return 1
  python tools/rocpd_timeline.py $(ls $d/*.db) --after cnn_fwd --skip 150 --count 24 --title "timeline, $name B=$B (PDM_FORCE_COMM=1 $*)" > $O/timeline_${name}_$B.md || return 1
  rm -rf $d
}
for B in ${XC_BATCHES:-256 32}; do
  one nocarry $B PDM_COMM=rccl PDM_RCCL_MODE=nocarry || exit 1
  one xgmi_xchg $B PDM_COMM=xgmi || exit 1
  one xgmi_stream $B PDM_COMM=xgmi PDM_XGMI_XCHG=0 || exit 1
done
echo done >> $O/bench.jsonl

# The fc1 update carried into the next forward launch (kernels/fc_carry.h) against the
# optimizer-run update, on the world-size>1 chain at N = 1 (PDM_FORCE_COMM=1): RCCL nocarry and
# xgmi, B = 256 and 32, bench + in-step trace each, two reps.  -> gpurun_out/carry/
set -o pipefail
O=gpurun_out/carry
mkdir -p $O
: > $O/bench.log
export TMPDIR=/tmp PDM_FORCE_COMM=1
one() {   # tag B env...
  local tag=$1 B=$2; shift 2
  echo "== $tag B=$B $*" >> $O/bench.log
  env "$@" timeout -k 10 150 python bench.py --scaling weak --batch-per-rank $B >> $O/bench.log 2>> $O/bench.err || return 1
  local d=$O/tr_${tag}_$B
  env "$@" timeout -k 10 150 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --scaling weak --batch-per-rank $B --steps 200 --warmup 30 > /dev/null 2>> $O/bench.err || return 1
  python tools/rocpd_summary.py $(ls $d/*.db) --title "$tag B=$B ($*)" --steps 150 > $O/${tag}_$B.md || return 1
  rm -rf $d
}
for rep in 1 2; do
  for B in 256 32; do
    one r${rep}_nocarry_carry $B PDM_COMM=rccl PDM_RCCL_MODE=nocarry || exit 1
    one r${rep}_nocarry_opt $B PDM_COMM=rccl PDM_RCCL_MODE=nocarry PDM_FC1_CARRY_FWD=0 || exit 1
    one r${rep}_xgmi_carry $B PDM_COMM=xgmi || exit 1
    one r${rep}_xgmi_opt $B PDM_COMM=xgmi PDM_FC1_CARRY_FWD=0 || exit 1
  done
done
echo done >> $O/bench.log

# bash tools/gpu_env_ab_args.sh NAME "bench args" "ENV=.. ENV2=.." ... : interleaved A/B of knob
# settings (the defaults are the first variant) on one bench.py configuration: the bench and an
# in-step rocprofv3 kernel trace per variant, twice.  -> gpurun_out/ab_NAME.log, ab_NAME_prof/
set -o pipefail
NAME=$1; ARGS=$2; shift 2
L=gpurun_out/ab_$NAME.log
P=gpurun_out/ab_${NAME}_prof
mkdir -p $P
: > $L
export TMPDIR=/tmp
for rep in 1 2; do
for v in "" "$@"; do
  tag=$(echo "${v:-default}" | tr ' =/' '___')
  echo "== rep $rep variant ${v:-default} $ARGS" >> $L
  env $v timeout -k 10 150 python bench.py $ARGS >> $L 2>&1 || exit 1
  d=$P/${rep}_${tag}
  env $v timeout -k 10 180 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py $ARGS --steps 200 --warmup 30 > /dev/null 2>&1 || exit 1
  python tools/rocpd_summary.py $(ls $d/*.db | head -1) --title "rep $rep ${v:-default} $ARGS" --steps 150 > ${d}.md && rm -rf $d
done
done
echo rc=$?

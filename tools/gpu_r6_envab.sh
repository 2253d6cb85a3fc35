# bash tools/gpu_r6_envab.sh NAME "VAR=val ..." "bench args;bench args;..." [reps]: interleaved A/B
# of an environment setting (A = without, B = with) over several bench.py configurations, and
# one in-step trace of the first configuration per variant.  -> gpurun_out/NAME/
set -o pipefail
name=$1; envs=$2; cfgs=$3; reps=${4:-2}
O=gpurun_out/$name
mkdir -p $O
export TMPDIR=/tmp
: > $O/ab.jsonl
IFS=';' read -ra CF <<< "$cfgs"
for rep in $(seq 1 $reps); do
  for v in A B; do
    for c in "${CF[@]}"; do
      echo "## rep=$rep $v $c" >> $O/ab.jsonl
      if [ $v = B ]; then env $envs timeout -k 10 150 python bench.py $c >> $O/ab.jsonl 2>> $O/bench.err || exit 1
      else timeout -k 10 150 python bench.py $c >> $O/ab.jsonl 2>> $O/bench.err || exit 1; fi
    done
    if [ $rep = 1 ]; then
      t=$O/tr_$v
      if [ $v = B ]; then env $envs timeout -k 10 150 rocprofv3 --kernel-trace -d $t -o run -- python3 bench.py ${CF[0]} --steps 200 --warmup 30 > /dev/null 2>&1 || exit 1
      else timeout -k 10 150 rocprofv3 --kernel-trace -d $t -o run -- python3 bench.py ${CF[0]} --steps 200 --warmup 30 > /dev/null 2>&1 || exit 1; fi
      python tools/rocpd_summary.py $(ls $t/*.db) --title "$v ($envs if B): bench.py ${CF[0]}" --steps 150 > $O/trace_$v.md; rm -rf $t
    fi
  done
done
python tools/refresh_summary.py $O/ab.jsonl > $O/ab_table.md
echo done

# bash tools/gpu_r6_multi.sh NAME "SO1 SO2 ..." "bench args;bench args;..." [reps]: interleaved
# bench.py runs of several builds of the extension (PDM_EXT_PATH; "-" = the in-tree build) over
# several configurations, plus one in-step kernel trace of the first configuration per build.
# -> gpurun_out/NAME/
set -o pipefail
name=$1; sos=$2; cfgs=$3; reps=${4:-2}
O=gpurun_out/$name
mkdir -p $O
export TMPDIR=/tmp
: > $O/ab.jsonl
IFS=';' read -ra CF <<< "$cfgs"
for rep in $(seq 1 $reps); do
  i=0
  for so in $sos; do
    i=$((i + 1))
    for c in "${CF[@]}"; do
      echo "## rep=$rep v$i $so $c" >> $O/ab.jsonl
      if [ "$so" = - ]; then timeout -k 10 150 python bench.py $c >> $O/ab.jsonl 2>> $O/bench.err || exit 1
      else PDM_EXT_PATH=$so timeout -k 10 150 python bench.py $c >> $O/ab.jsonl 2>> $O/bench.err || exit 1; fi
    done
    if [ $rep = 1 ]; then
      t=$O/tr_v$i
      if [ "$so" = - ]; then timeout -k 10 150 rocprofv3 --kernel-trace -d $t -o run -- python3 bench.py ${CF[0]} --steps 200 --warmup 30 > /dev/null 2>&1 || exit 1
      else PDM_EXT_PATH=$so timeout -k 10 150 rocprofv3 --kernel-trace -d $t -o run -- python3 bench.py ${CF[0]} --steps 200 --warmup 30 > /dev/null 2>&1 || exit 1; fi
      python tools/rocpd_summary.py $(ls $t/*.db) --title "v$i ($so): bench.py ${CF[0]}" --steps 150 > $O/trace_v$i.md; rm -rf $t
    fi
  done
done
python tools/refresh_summary.py $O/ab.jsonl > $O/ab_table.md
echo done

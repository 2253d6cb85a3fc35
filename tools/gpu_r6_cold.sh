# First-launch vs chip-idle windows (tools/graph_gaps.py) and two kernel traces of bench.py's
# driver window (idle gaps inside it).  bash tools/gpu_r6_cold.sh NAME
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/graph_gaps.py 5 > $O/gaps.txt 2>&1 || exit 1
for r in 1 2; do
  t=$O/tr$r
  timeout -k 10 150 rocprofv3 --kernel-trace -d $t -o run -- python3 bench.py --steps 20 --warmup 5 > $O/bench_tr$r.log 2>&1 || exit 1
  db=$(ls $t/*/*.db $t/*.db 2>/dev/null | head -1)
  python tools/rocpd_timeline.py $db --last 200 --count 200 --title "driver window $r" > $O/timeline$r.md
  rm -rf $t
done
cat $O/gaps.txt

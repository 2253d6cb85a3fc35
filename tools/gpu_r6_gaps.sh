# tools/graph_gaps.py timed plainly and under a kernel trace (gaps per window): bash tools/gpu_r6_gaps.sh NAME
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/graph_gaps.py 7 > $O/g8.txt 2>&1 || exit 1
t=$O/tr
timeout -k 10 200 rocprofv3 --kernel-trace -d $t -o run -- python3 tools/graph_gaps.py 5 > $O/g8_traced.txt 2>&1 || exit 1
db=$(ls $t/*/*.db $t/*.db 2>/dev/null | head -1)
(cd tools && python gaps_from_trace.py ../$db full20 split tail boundary boundary_pf) > $O/gaps.txt 2>&1
cp $db $O/run.db; rm -rf $t
cat $O/g8.txt $O/gaps.txt

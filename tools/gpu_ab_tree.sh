# bash tools/gpu_ab_tree.sh NAME "BENCH ARGS" build/wt_a [build/wt_b ...]
# Interleaved A/B of whole trees: each variant is a git worktree under build/ with its own
# Python and in-tree extension (git worktree add build/wt_x <commit> && (cd build/wt_x &&
# python -m pytorch_distributed_mnist_amd.build)), so Python-side changes are compared too;
# the current tree is the last variant.  bench.py twice per variant, interleaved, and one
# in-step rocprofv3 kernel trace per variant summarised on the box -> gpurun_out/NAME/.
set -o pipefail
name=$1; args=$2; shift 2
O=gpurun_out/$name
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
: > $O/ab.jsonl
for rep in 1 2; do
  for v in "$@" tree; do
    tag=$(basename $v)
    echo "## rep=$rep $tag" >> $O/ab.jsonl
    if [ $v = tree ]; then d=$R; else d=$R/$v; fi
    ( cd $d && timeout -k 10 150 python bench.py $args ) >> $O/ab.jsonl 2>> $O/bench.err || exit 1
    if [ $rep = 1 ]; then
      t=$R/$O/tr_$tag
      ( cd $d && timeout -k 10 150 rocprofv3 --kernel-trace -d $t -o run -- python3 bench.py $args > /dev/null 2>&1 ) || exit 1
      python tools/rocpd_summary.py $(ls $t/*.db) --title "$tag: bench.py $args" --steps 80 > $O/trace_$tag.md; rm -rf $t
    fi
  done
done
python tools/refresh_summary.py $O/ab.jsonl > $O/ab_table.md
echo done

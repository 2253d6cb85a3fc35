set -o pipefail
O=gpurun_out/r4j
mkdir -p $O
export TMPDIR=/tmp
: > $O/check.txt
for B in 64 256; do
  for u in "" 1 6; do
    PDM_F32_UPW=$u timeout -k 10 120 python tools/f32_grad_check.py $B x3 >> $O/check.txt 2>&1 || exit 1
  done
done
timeout -k 10 120 python tools/f32_grad_check.py 64 exact >> $O/check.txt 2>&1 || exit 1
echo done

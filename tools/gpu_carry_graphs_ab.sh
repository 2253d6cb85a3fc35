# The carried fc1 update across graph replays (StepStructure.fc1_carry_graphs) against carrying
# it within each 8-step graph only: forced N = 1, xgmi and RCCL nocarry, B = 256 / 32, two reps.
set -o pipefail
O=gpurun_out/carryg
mkdir -p $O
: > $O/bench.log
export PDM_FORCE_COMM=1
for rep in 1 2; do for B in 256 32; do
  for t in "PDM_COMM=xgmi" "PDM_COMM=rccl PDM_RCCL_MODE=nocarry"; do for g in 1 0; do
    echo "== rep $rep B=$B $t PDM_FC1_CARRY_GRAPHS=$g" >> $O/bench.log
    env $t PDM_FC1_CARRY_GRAPHS=$g timeout -k 10 150 python bench.py --scaling weak --batch-per-rank $B >> $O/bench.log 2>> $O/bench.err || exit 1
  done; done
done; done
echo done >> $O/bench.log

#!/bin/bash
# PMC counter passes over tools/step_loop.py (eager steps), one rocprofv3 run per pass
# (counter slots per pass: MI355X_MICROARCH.md "rocprofv3 PMC slots"), plus a kernel-trace
# run for durations, then the derived per-kernel table (tools/pmc_table.py).
#   bash tools/pmc_run.sh NAME B DTYPE [force|local] [seq]   -> gpurun_out/pmc/NAME/*, NAME.md
# (seq: the 30 steps as one train_steps call, tools/step_loop.py)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
name=${1:-b256}; B=${2:-256}; DT=${3:-bf16}; FORCE=${4:-}; SEQ=${5:-}
out=gpurun_out/pmc/$name
mkdir -p "$out"
prog="python3 tools/step_loop.py $B 30 $DT ${FORCE:-local} $SEQ"
pass() {
  local p=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$out/$p" -o run \
    -- $prog > "$out/$p.log" 2>&1
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE
pass st SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES
pass rd FETCH_SIZE
pass wr WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$out/trace" -o run \
  -- $prog > "$out/trace.log" 2>&1
python3 tools/pmc_table.py --title "$name: eager steps${SEQ:+ (one train_steps call)}, B=$B, $DT $FORCE (30 steps, means per dispatch)" \
  --trace "$out/trace" "$out/sq" "$out/st" "$out/rd" "$out/wr" > gpurun_out/pmc/$name.md

#!/bin/bash
# Instruction-mix / stall PMC passes over tools/step_loop.py (eager CNN steps, B=256): where a
# kernel's wave cycles go (VALU vs MFMA vs LDS issue, LDS waits).  One rocprofv3 run per pass.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/pmcb
mkdir -p "$out"
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run \
    -- python3 tools/step_loop.py 256 30 > "$out/$name.log" 2>&1
}
pass a SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY
pass b SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU_CVT
python3 tools/pmc_summary.py $(find "$out" -name '*counter_collection.csv') > gpurun_out/pmcb.md

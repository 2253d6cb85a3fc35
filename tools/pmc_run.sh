#!/bin/bash
# PMC counter passes over tools/step_loop.py (eager CNN steps, B=256), one rocprofv3 run per
# pass (counter slots per pass: MI355X_MICROARCH.md "rocprofv3 PMC slots"), then a table.
# Run on the GPU box:  bash tools/pmc_run.sh  -> gpurun_out/pmc/*, gpurun_out/pmc.md
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/pmc
mkdir -p "$out"
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run \
    -- python3 tools/step_loop.py 256 30 > "$out/$name.log" 2>&1
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE
pass rd FETCH_SIZE GRBM_COUNT
pass wr WRITE_SIZE TCC_HIT_sum
python3 tools/pmc_summary.py $(find "$out" -name '*counter_collection.csv') > gpurun_out/pmc.md

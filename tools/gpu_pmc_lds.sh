# One PMC pass: LDS bank-conflict cycles vs LDS active cycles per kernel (B=256 eager steps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcl
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS --output-format csv -d gpurun_out/pmcl/a -o run -- python3 tools/step_loop.py 256 30 > gpurun_out/pmcl/a.log 2>&1 && \
python3 tools/pmc_summary.py $(find gpurun_out/pmcl -name '*counter_collection.csv') > gpurun_out/pmcl.md
echo rc=$?

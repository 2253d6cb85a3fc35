mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 5 60 rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1; echo rc=$?

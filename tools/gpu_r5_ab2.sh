# fc1_bwd at two workgroups per CU (<= 256 registers) vs the default, local chain B = 256 / 32;
# then the persistent xgmi collective's width / unroll at N = 1 forced, B = 32.
set -o pipefail
bash tools/gpu_ab_b.sh "256 32" build/fcw2 || exit 1
mv gpurun_out/abb.log gpurun_out/ab_fc.log && rm -rf gpurun_out/ab_fc_prof && mv gpurun_out/abb_prof gpurun_out/ab_fc_prof || exit 1
PDM_FORCE_COMM=1 PDM_COMM=xgmi bash tools/gpu_ab_b.sh "32" build/xg128 build/xgu8 || exit 1
mv gpurun_out/abb.log gpurun_out/ab_xg.log && rm -rf gpurun_out/ab_xg_prof && mv gpurun_out/abb_prof gpurun_out/ab_xg_prof

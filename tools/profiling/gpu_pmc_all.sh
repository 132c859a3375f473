# HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the dominant kernel of each
# bench workload -> gpurun_out/pmc_traffic_<algo>.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
for pair in ${PAIRS:-td3bc:gemm_rd_kernel bcq:mlp_fwd_kernel dcql:conv_fwd_kernel cqldp:mlp_fwd_kernel}; do
  a=${pair%%:*}; k=${pair#*:}
  bash $R/tools/profiling/pmc_pass.sh $a $k || exit $?
  cd $R && find gpurun_out/pmc_fetch_$a gpurun_out/pmc_write_$a -name "*.csv" -size +20M -delete
done

# BASELINE.md CPU protocol for K1 (td3bc), K4 (cqldp), K3 (bcq), K5 (dcql) on
# the GPU box's host (no GPU used).  Step counts are bounded per algorithm so
# the whole call stays within ~15 minutes; every leg's step count is recorded.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
P="python3 -u tools/cpu_baseline_protocol.py --sweep 1,16,64,128 --sweep-seconds 8"
timeout -k 10 240 $P --algo td3bc --steps 1000 --warmup 50 --runs 5 --phys-steps 200 --phys-runs 3 --out gpurun_out/r03_cpu_baseline_td3bc.json > gpurun_out/r03_cpu_baseline_td3bc.log 2>&1 || exit $?
timeout -k 10 360 $P --algo cqldp --steps 300 --warmup 20 --runs 5 --phys-steps 20 --phys-runs 3 --out gpurun_out/r03_cpu_baseline_cqldp.json > gpurun_out/r03_cpu_baseline_cqldp.log 2>&1 || exit $?
timeout -k 10 360 $P --algo bcq --steps 50 --warmup 5 --runs 5 --phys-steps 5 --phys-runs 3 --out gpurun_out/r03_cpu_baseline_bcq.json > gpurun_out/r03_cpu_baseline_bcq.log 2>&1 || exit $?
timeout -k 10 360 $P --algo dcql --steps 30 --warmup 3 --runs 5 --phys-steps 3 --phys-runs 3 --out gpurun_out/r03_cpu_baseline_dcql.json > gpurun_out/r03_cpu_baseline_dcql.log 2>&1

# CPU protocol for K1 (td3bc) and K4 (cqldp) in one call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python3 -u tools/cpu_baseline_protocol.py --algo td3bc --steps 1000 --warmup 50 --runs 5 --sweep 1,16,64,128 --sweep-seconds 8 --phys-steps 200 --phys-runs 3 --out gpurun_out/r03_cpu_baseline_td3bc.json > gpurun_out/r03_cpu_baseline_td3bc.log 2>&1 || exit $?
timeout -k 10 600 python3 -u tools/cpu_baseline_protocol.py --algo cqldp --steps 300 --warmup 20 --runs 5 --sweep 1,16,64,128 --sweep-seconds 8 --phys-steps 20 --phys-runs 3 --out gpurun_out/r03_cpu_baseline_cqldp.json > gpurun_out/r03_cpu_baseline_cqldp.log 2>&1

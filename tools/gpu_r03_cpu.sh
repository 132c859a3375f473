# BASELINE.md CPU protocol on the GPU box's host: $1 algo, $2 steps, $3 runs,
# $4 sweep list, $5 warmup, $6 physical-cores steps, $7 physical-cores runs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 1100 python3 -u tools/cpu_baseline_protocol.py --algo $1 --steps $2 --warmup $5 --runs $3 --sweep "$4" --sweep-seconds 10 --phys-steps $6 --phys-runs $7 --out gpurun_out/r03_cpu_baseline_$1.json > gpurun_out/r03_cpu_baseline_$1.log 2>&1

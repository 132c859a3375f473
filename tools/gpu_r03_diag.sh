set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python3 tools/diag_k4.py > gpurun_out/diag_k4.log 2>&1

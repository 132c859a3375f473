# Quick health run of the committed tree: GPU suite + K2 bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -q -x -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/q_gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 2000 > gpurun_out/q_bench_cql.log 2>&1 || exit $?

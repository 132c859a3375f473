# The Adam / partial-reduction kernel tests alone.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -q -x -m gpu -k adam -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/adam_tests.log 2>&1; rc=$?; tail -15 gpurun_out/adam_tests.log; exit $rc

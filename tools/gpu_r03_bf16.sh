# bf16 critic kernels: tests, then a short bf16 bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/bf16_tests.log 2>&1; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
true

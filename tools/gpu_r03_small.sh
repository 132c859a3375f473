# small-pass MLP kernel: its tests, the parity suites whose policies / targets
# now run on it, then the K2 iteration run (bench + kernel trace).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "mlp" tests/test_gpu_td3_parity.py tests/test_gpu_bcq_parity.py tests/test_gpu_sac_parity.py -q -x -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/small_tests.log 2>&1 || exit $?
TESTS="tests/test_gpu_cql_parity.py tests/test_gpu_production_path.py" bash tools/gpu_r03_iter.sh

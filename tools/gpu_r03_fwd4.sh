set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
bash tools/gpu_r03_fwd3.sh || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "fused_mlp" -q -x -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/fwd2_tests.log 2>&1 || exit $?
TESTS="tests/test_gpu_cql_parity.py tests/test_gpu_production_path.py" bash tools/gpu_r03_iter.sh

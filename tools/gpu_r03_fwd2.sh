# q2_fwd A/B on the K2 shape, the fused-forward tests, then the iteration run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 120 python3 tools/bench_fwd.py > gpurun_out/fwd2_bench.json 2>gpurun_out/fwd2_bench.err || exit $?
D3A_FWD_Q2=0 timeout -k 10 120 python3 tools/bench_fwd.py >> gpurun_out/fwd2_bench.json 2>>gpurun_out/fwd2_bench.err || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "fused_mlp" -q -x -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/fwd2_tests.log 2>&1 || exit $?
TESTS="tests/test_gpu_cql_parity.py tests/test_gpu_production_path.py" bash tools/gpu_r03_iter.sh

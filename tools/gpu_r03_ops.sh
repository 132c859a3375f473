# torch custom-op tests + q2 kernel test / microbench.  Outputs in gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_torch_ops.py tests/test_gpu_torch_modules.py tests/test_gpu_q2_bwd.py -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ops_tests.log 2>&1; rc=$?
timeout -k 10 120 python3 tools/bench_q2.py > gpurun_out/q2_bench.json 2>gpurun_out/q2_bench.err || exit $?
exit $rc

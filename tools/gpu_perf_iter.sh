# perf iteration: K2 parity-critical tests, then K2 bench + one-step timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread ${TESTS:-tests/test_gpu_cql_parity.py tests/test_gpu_kernels.py tests/test_gpu_dp.py tests/test_gpu_production_path.py} > gpurun_out/it_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 2000 --no-cpu-baseline > gpurun_out/it_bench.log 2>&1 || exit $?
bash tools/gpu_timeline.sh

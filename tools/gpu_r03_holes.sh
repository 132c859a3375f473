set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "tests/test_gpu_production_path.py::test_cql_fit_production_path_per_step_proof" -v -s -m gpu -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/holes_tests.log 2>&1

# full GPU suite + smoke (round validation); outputs in gpurun_out/
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/full_gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 || exit $?

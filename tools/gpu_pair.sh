# Paired backward GEMMs: bit-identity test, then the iteration check (suite, benches, timeline).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -q -x -m gpu -k "gemm_pair" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pair_tests.log 2>&1 || { tail -40 gpurun_out/pair_tests.log; exit 1; }
tail -1 gpurun_out/pair_tests.log
bash tools/gpu_iter2.sh

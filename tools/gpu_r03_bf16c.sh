set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
: > gpurun_out/bf16c.json
for p in 0 2 8 16 24; do
  D3A_BF16_PROBE=$p timeout -k 10 120 python3 tools/bench_bf16.py >> gpurun_out/bf16c.json 2>>gpurun_out/bf16c.err || exit $?
done
timeout -k 10 120 python3 tools/bench_fwd.py --bf16 >> gpurun_out/bf16c.json 2>>gpurun_out/bf16c.err || exit $?
timeout -k 10 120 python3 tools/bench_fwd.py >> gpurun_out/bf16c.json 2>>gpurun_out/bf16c.err || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -q -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/bf16_tests.log 2>&1 || exit $?

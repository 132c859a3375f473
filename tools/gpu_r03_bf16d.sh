set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
: > gpurun_out/bf16d.json
timeout -k 10 120 python3 tools/bench_fwd.py --bf16 >> gpurun_out/bf16d.json 2>>gpurun_out/bf16d.err || exit $?
timeout -k 10 120 python3 tools/bench_bf16.py >> gpurun_out/bf16d.json 2>>gpurun_out/bf16d.err || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -q -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/bf16_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --precision bf16 > gpurun_out/bench_bf16.json 2>gpurun_out/bench_bf16.err || exit $?

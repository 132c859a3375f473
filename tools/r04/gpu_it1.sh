# r04 iteration 1: parity-arbiter tests, actor_q fix, x6 forward kernel + microbench
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_x6.py > gpurun_out/it1_x6.log 2>&1 || exit $?
timeout -k 10 120 python tools/bench_fwd.py --x6 > gpurun_out/it1_fwd.jsonl 2>&1 || exit $?
timeout -k 10 120 python tools/bench_fwd.py >> gpurun_out/it1_fwd.jsonl 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_actor_q.py tests/test_gpu_dp.py tests/test_gpu_production_path.py > gpurun_out/it1_tests.log 2>&1

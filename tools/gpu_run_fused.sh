set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -q -x -m gpu -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 --no-cpu-baseline > gpurun_out/b_cql.log 2>&1 || exit $?
D3A_FUSED_BWD=1 timeout -k 10 300 python bench.py --steps 2000 --warmup 50 --no-cpu-baseline > gpurun_out/b_cql_fbwd.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --algo bcq --steps 500 --warmup 20 --no-cpu-baseline > gpurun_out/b_bcq.log 2>&1 || exit $?
D3A_FUSED_BWD=1 timeout -k 10 300 python bench.py --algo bcq --steps 500 --warmup 20 --no-cpu-baseline > gpurun_out/b_bcq_fbwd.log 2>&1 || exit $?

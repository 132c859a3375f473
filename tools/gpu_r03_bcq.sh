# BCQ target-kernel change: BCQ / arbiter GPU tests, K3 bench line, K3 kernel breakdown.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_bcq_parity.py tests/test_gpu_arbiters.py tests/test_gpu_torch_modules.py > gpurun_out/bcq_tests.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --algo bcq --no-cpu-baseline > gpurun_out/bcq_bench.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/bcq_prof -o run --output-format csv -- python3 bench.py --algo bcq --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/bcq_prof.log 2>&1 || exit $?
f=$(find gpurun_out/bcq_prof -name '*kernel_trace.csv' -print -quit)
python tools/prof_by_shape.py "$f" 70 > gpurun_out/bcq_breakdown.txt 2>&1 || true
rm -f "$f"

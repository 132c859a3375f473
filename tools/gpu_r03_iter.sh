# Round-3 iteration run: the new kernels' tests, the CQL parity set, a K2
# bench line and a kernel-trace of a short K2 bench.  Outputs in gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T="${TESTS:-tests/test_gpu_q2_bwd.py tests/test_gpu_cql_parity.py tests/test_gpu_production_path.py tests/test_gpu_dp.py}"
timeout -k 10 400 python -u -m pytest $T -q -x -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/it_tests.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 2000 --no-cpu-baseline > gpurun_out/it_bench_cql.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/it_prof -o it --output-format csv -- python3 bench.py --steps 300 --warmup 20 --no-cpu-baseline --transitions 200000 > gpurun_out/it_prof.log 2>&1 || exit $?
f=$(find gpurun_out/it_prof -name '*kernel_trace.csv' -print -quit)
python tools/prof_by_shape.py "$f" 320 > gpurun_out/it_breakdown.txt 2>&1 || true
python tools/prof_timeline.py "$f" > gpurun_out/it_timeline.txt 2>&1 || true

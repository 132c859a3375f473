# Actor-phase critic kernel (d3a_sac_actor_q): its tests, the CQL / SAC / DP /
# production-path parity suites, K2 bench lines with and without it, timeline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_actor_q.py tests/test_gpu_cql_parity.py tests/test_gpu_sac_parity.py tests/test_gpu_production_path.py tests/test_gpu_dp.py > gpurun_out/aq_tests.log 2>&1 || exit $?
timeout -k 10 120 python bench.py --steps 2000 --no-cpu-baseline > gpurun_out/aq_bench.log 2>&1 || exit $?
D3A_ACTOR_Q=0 timeout -k 10 120 python bench.py --steps 2000 --no-cpu-baseline > gpurun_out/aq_bench_off.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/aq_prof -o k2 --output-format csv -- python3 bench.py --steps 300 --warmup 20 --no-cpu-baseline --transitions 200000 > gpurun_out/aq_prof.log 2>&1 || exit $?
f=$(find gpurun_out/aq_prof -name '*kernel_trace.csv' -print -quit)
python tools/prof_timeline.py "$f" > gpurun_out/aq_timeline.txt 2>&1 || true
rm -f "$f"

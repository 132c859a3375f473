# Policy forward over unit parts (d3a_mlp_fwd parts): kernel tests, the CQL /
# SAC / DP / production-path parity suites, K2 bench with and without, timeline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_actor_q.py tests/test_gpu_cql_parity.py tests/test_gpu_sac_parity.py tests/test_gpu_production_path.py tests/test_gpu_dp.py > gpurun_out/pt_tests.log 2>&1 || exit $?
timeout -k 10 120 python bench.py --steps 2000 --no-cpu-baseline > gpurun_out/pt_bench.log 2>&1 || exit $?
D3A_MLP_PARTS=0 timeout -k 10 120 python bench.py --steps 2000 --no-cpu-baseline > gpurun_out/pt_bench_off.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pt_prof -o k2 --output-format csv -- python3 bench.py --steps 300 --warmup 20 --no-cpu-baseline --transitions 200000 > gpurun_out/pt_prof.log 2>&1 || exit $?
f=$(find gpurun_out/pt_prof -name '*kernel_trace.csv' -print -quit)
python tools/prof_timeline.py "$f" > gpurun_out/pt_timeline.txt 2>&1 || true
rm -f "$f"

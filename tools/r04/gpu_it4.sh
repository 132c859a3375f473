# r04 iteration 4: x6 v2 kernels (64-unit chunks / role-split staging): tests, benches, probes;
# CQL parity + production path with the x6 critic GEMMs
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_x6.py > gpurun_out/r4i4_x6.log 2>&1 || exit $?
for p in 0 1 4 7; do D3A_X6_PROBE=$p timeout -k 10 120 python tools/bench_fwd.py --x6 | sed "s/^/fwd probe $p: /" >> gpurun_out/r4i4_probe.txt 2>/dev/null || exit $?; done
for p in 0 8 16 32 56; do D3A_X6_PROBE=$p timeout -k 10 120 python tools/bench_q2.py --x6 | sed "s/^/bwd probe $p: /" >> gpurun_out/r4i4_probe.txt 2>/dev/null || exit $?; done
timeout -k 10 200 python bench.py --critic-gemm x6 --no-cpu-baseline >> gpurun_out/r4i4_bench.jsonl 2>/dev/null || exit $?
D3A_CRITIC_GEMM=x6 timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_production_path.py tests/test_gpu_cql_parity.py tests/test_gpu_dp.py > gpurun_out/r4i4_tests_x6.log 2>&1

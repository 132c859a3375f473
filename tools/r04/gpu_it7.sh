# r04 iteration 7: restructured x6 forward (split production, pipelined B reads): test, stamps, probes, CQL parity both modes
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_x6.py > gpurun_out/r4i7_x6.log 2>&1 || exit $?
timeout -k 10 120 python tools/x6_stamps.py > gpurun_out/r4i7_stamps.txt 2>&1 || exit $?
for p in 0 4 1; do D3A_X6_PROBE=$p timeout -k 10 120 python tools/bench_fwd.py --x6 | sed "s/^/fwd probe $p: /" >> gpurun_out/r4i7_probe.txt 2>/dev/null || exit $?; done
D3A_CRITIC_GEMM=x6 timeout -k 10 900 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread -m gpu tests/test_gpu_cql_parity.py > gpurun_out/r4i7_parity_x6.log 2>&1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread -m gpu tests/test_gpu_cql_parity.py > gpurun_out/r4i7_parity_fp32.log 2>&1

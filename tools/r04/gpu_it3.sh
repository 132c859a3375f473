# r04 iteration 3: x6 kernel probe sweep (timing only) + CQL parity (repro arbiter) + GC capture test
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
for p in 0 1 2 4 7; do D3A_X6_PROBE=$p timeout -k 10 120 python tools/bench_fwd.py --x6 | sed "s/^/fwd probe $p: /" >> gpurun_out/r4i3_probe.txt 2>/dev/null || exit $?; done
for p in 0 8 16 32 56; do D3A_X6_PROBE=$p timeout -k 10 120 python tools/bench_q2.py --x6 | sed "s/^/bwd probe $p: /" >> gpurun_out/r4i3_probe.txt 2>/dev/null || exit $?; done
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_capture_gc.py tests/test_gpu_cql_parity.py > gpurun_out/r4i3_tests.log 2>&1

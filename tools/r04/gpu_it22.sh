# r04 iteration 22: conv input gradient on fp32 MFMA with packed weights (default)
# vs split-bf16: conv tests, K5 arbiter, microbench, K5 bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_conv.py > gpurun_out/i22_conv.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_arbiters.py tests/test_gpu_discrete_cql.py > gpurun_out/i22_arb.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for x in 1 0; do D3A_CONV_BWD_X_F32=$x timeout -k 10 120 python tools/bench_conv_bwd.py | sed "s/^/f32 $x: /" >> gpurun_out/i22_convbench.txt 2>gpurun_out/i22_convbench.err || exit $?; done
for x in 1 0; do D3A_CONV_BWD_X_F32=$x timeout -k 10 300 python bench.py --algo dcql --steps 300 --warmup 20 --no-cpu-baseline | sed "s/^/f32 $x: /" >> gpurun_out/i22_bench.txt 2>/dev/null || exit $?; done

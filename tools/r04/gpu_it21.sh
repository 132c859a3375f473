# r04 iteration 21: which K5 change moves the B=512 arbiter's conv gradients
# (conv input gradient vs fc split-bf16), packed-weight conv input gradient
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_conv.py -k bwd_x > gpurun_out/i21_conv.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for v in "D3A_CONV_BWD_X=0" "D3A_FC_SPLITK=0" "D3A_CONV_BWD_X6=0"; do
  env $v timeout -k 10 300 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_arbiters.py -k k5_b512 > gpurun_out/i21_arb_$v.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
done
timeout -k 10 120 python tools/bench_conv_bwd.py > gpurun_out/i21_convbench.jsonl 2>gpurun_out/i21_convbench.err || exit $?
timeout -k 10 300 python bench.py --algo dcql --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/i21_bench.txt 2>/dev/null || exit $?
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_conv.py > gpurun_out/i22_conv.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_arbiters.py tests/test_gpu_discrete_cql.py > gpurun_out/i22_arb.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for x in 1 0; do D3A_CONV_BWD_X_F32=$x timeout -k 10 120 python tools/bench_conv_bwd.py | sed "s/^/f32 $x: /" >> gpurun_out/i22_convbench.txt 2>gpurun_out/i22_convbench.err || exit $?; done
for x in 1 0; do D3A_CONV_BWD_X_F32=$x timeout -k 10 300 python bench.py --algo dcql --steps 300 --warmup 20 --no-cpu-baseline | sed "s/^/f32 $x: /" >> gpurun_out/i22_bench.txt 2>/dev/null || exit $?; done

# r04 iteration 11: x6 backward with quarter-restricted head sums: kernel tests,
# microbench, K2 benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -s -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_x6.py tests/test_gpu_q2_bwd.py > gpurun_out/i11_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for p in 0 8; do D3A_X6_PROBE=$p timeout -k 10 120 python tools/bench_q2.py --x6 | sed "s/^/bwd probe $p: /" >> gpurun_out/i11_probe.txt 2>/dev/null || exit $?; done
for sw in "20 5" "2000 50"; do set -- $sw; timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-cpu-baseline >> gpurun_out/i11_bench.jsonl 2>/dev/null || exit $?; done

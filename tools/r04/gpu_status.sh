# r04 re-entry status: full GPU suite (fp32 critic GEMMs), the CQL suites with the x6
# critic kernels, smoke(), and bench lines for fp32 / x6 / the reproduction config
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/st_gpu_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
D3A_CRITIC_GEMM=x6 timeout -k 10 600 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_x6.py tests/test_gpu_cql_parity.py tests/test_gpu_production_path.py tests/test_gpu_dp.py tests/test_gpu_arbiters.py tests/test_gpu_bcq_parity.py > gpurun_out/st_gpu_tests_x6.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/st_smoke.log 2>&1 || exit $?
for g in fp32 x6; do timeout -k 10 200 python bench.py --critic-gemm $g --no-cpu-baseline >> gpurun_out/st_bench.jsonl 2>>gpurun_out/st_bench.err || exit $?; done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/st_bench.jsonl 2>>gpurun_out/st_bench.err || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --critic-gemm x6 --no-cpu-baseline >> gpurun_out/st_bench.jsonl 2>>gpurun_out/st_bench.err || exit $?
for a in cqlrepro bcq; do for g in fp32 x6; do timeout -k 10 200 python bench.py --algo $a --critic-gemm $g --no-cpu-baseline >> gpurun_out/st_bench.jsonl 2>>gpurun_out/st_bench.err || exit $?; done; done
for o in 0 1; do D3A_FWDB_OLD=$o timeout -k 10 120 python tools/bench_bf16.py | sed "s/^/bf16 old=$o: /" >> gpurun_out/st_bf16.txt 2>/dev/null || exit $?; done
for o in 0 1; do D3A_FWDB_OLD=$o timeout -k 10 200 python bench.py --precision bf16 --no-cpu-baseline >> gpurun_out/st_bench.jsonl 2>>gpurun_out/st_bench.err || exit $?; done

# Iteration check: GPU suite, the five bench lines, the K2 per-launch timeline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -q -x -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/it_tests.log 2>&1 || { tail -30 gpurun_out/it_tests.log; exit 1; }
tail -1 gpurun_out/it_tests.log
for a in cql td3bc cqldp bcq dcql; do
  timeout -k 10 200 python bench.py --algo $a --steps 2000 --no-cpu-baseline > gpurun_out/it_bench_$a.log 2>&1 || exit $?
  echo "$a $(grep -o '"value": [0-9.]*' gpurun_out/it_bench_$a.log)"
done
bash tools/gpu_timeline.sh && cat gpurun_out/tl_cql.txt

# A/B of the in-head dQ/da path (pairs threshold) on K2 and K4, plus the CQL/SAC parity tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
for a in cql cqldp; do
  for m in 0 8 32; do
    D3A_DQ_IN_HEAD_MAX_PAIRS=$m timeout -k 10 200 python bench.py --algo $a --steps 3000 --no-cpu-baseline > gpurun_out/ab_dq_${a}_$m.log 2>&1 || exit $?
    echo "$a pairs<=$m $(grep -o '"value": [0-9.]*' gpurun_out/ab_dq_${a}_$m.log)"
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_cql_parity.py tests/test_gpu_sac_parity.py tests/test_gpu_production_path.py tests/test_gpu_arbiters.py tests/test_gpu_dp.py -q -x -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab_dq_tests.log 2>&1 || { tail -30 gpurun_out/ab_dq_tests.log; exit 1; }
tail -1 gpurun_out/ab_dq_tests.log

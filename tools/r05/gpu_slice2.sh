#!/bin/bash
# round 5: slice backward parity (kernel + CQL suites) and the K2 bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5b
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_x6t.py tests/test_gpu_x6.py > gpurun_out/r5b/tests_kernel.log 2>&1
st=$?; tail -3 gpurun_out/r5b/tests_kernel.log; [ $st -ne 0 ] && exit $st
for m in rows slice; do
  timeout -k 10 120 python -u tools/bench_q2.py --x6 --mask $m >> gpurun_out/r5b/bench_q2.jsonl 2>&1 || exit $?
done
timeout -k 10 120 python -u tools/bench_q2.py --x6 --mask slice --n-in 37 >> gpurun_out/r5b/bench_q2.jsonl 2>&1 || exit $?
cat gpurun_out/r5b/bench_q2.jsonl
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_cql_parity.py tests/test_gpu_production_path.py tests/test_gpu_dp.py > gpurun_out/r5b/tests_cql.log 2>&1
st=$?; tail -3 gpurun_out/r5b/tests_cql.log; [ $st -ne 0 ] && exit $st
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 50 > gpurun_out/r5b/bench_k2.json 2> gpurun_out/r5b/bench_k2.err || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5b/bench_k2_20.json 2>> gpurun_out/r5b/bench_k2.err || exit $?
cat gpurun_out/r5b/bench_k2.json gpurun_out/r5b/bench_k2_20.json

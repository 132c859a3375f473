#!/bin/bash
# round 5: the slice critic backward (q2_x6_bwd2.hip) -- parity against fp64
# and launch time against the 256-row-block kernel on the K2 shape
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5a
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_x6t.py tests/test_gpu_x6.py > gpurun_out/r5a/tests.log 2>&1
st=$?
tail -5 gpurun_out/r5a/tests.log
[ $st -ne 0 ] && exit $st
for m in rows slice; do
  timeout -k 10 120 python -u tools/bench_q2.py --x6 --mask $m >> gpurun_out/r5a/bench.jsonl 2>&1 || exit $?
done
timeout -k 10 120 python -u tools/bench_q2.py --x6 --mask slice --n-in 37 >> gpurun_out/r5a/bench.jsonl 2>&1 || exit $?
cat gpurun_out/r5a/bench.jsonl

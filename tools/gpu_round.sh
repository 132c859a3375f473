#!/bin/bash
# One gpurun session: GPU tests, a bench line, and a rocprofv3 kernel-trace profile.
# Stops at the first abort / segfault / timeout (exit codes other than 0 and 1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out
mkdir -p $OUT
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
STEP=${1:-all}
if [ "$STEP" = all ] || [ "$STEP" = test ]; then
  timeout -k 10 ${TEST_TIMEOUT:-400} python -m pytest tests -q -s -m gpu -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log; ok $rc || exit $rc
fi
if [ "$STEP" = all ] || [ "$STEP" = bench ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:---steps 1000 --warmup 50} > $OUT/bench.log 2>&1
  rc=$?; echo "bench rc=$rc" >> $OUT/bench.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "$STEP" = all ] || [ "$STEP" = prof ]; then
  R=$(pwd)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats -d $R/$OUT/prof -o run --output-format csv -- python3 $R/bench.py ${PROF_ARGS:---steps 300 --warmup 20 --no-cpu-baseline --transitions 200000} > $R/$OUT/prof.log 2>&1
  rc=$?; echo "prof rc=$rc" >> $R/$OUT/prof.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0

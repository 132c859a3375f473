#!/bin/bash
# Run named GPU steps in order, each under its own time limit; stop at the
# first abort / segfault / timeout (exit codes other than 0 and 1 for tests).
#   bash tools/gpu_steps.sh test bench bench_td3 prof sweep
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out
mkdir -p $OUT
R=$(pwd)
for STEP in "$@"; do
  case $STEP in
    test)
      timeout -k 10 ${TEST_TIMEOUT:-500} python -m pytest tests -q -s -m gpu -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
      rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log; [ $rc -le 1 ] || exit $rc ;;
    bench)
      timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 2000 --warmup 50} > $OUT/bench.log 2>&1
      rc=$?; echo "bench rc=$rc" >> $OUT/bench.log; [ $rc -eq 0 ] || exit $rc ;;
    bench_td3)
      timeout -k 10 400 python bench.py --algo td3bc ${BENCH_TD3_ARGS:---steps 4000 --warmup 50 --transitions 100000} > $OUT/bench_td3.log 2>&1
      rc=$?; echo "bench rc=$rc" >> $OUT/bench_td3.log; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof -o run --output-format csv -- python3 $R/bench.py ${PROF_ARGS:---steps 300 --warmup 20 --no-cpu-baseline --transitions 200000} > $R/$OUT/prof.log 2>&1)
      rc=$?; echo "prof rc=$rc" >> $OUT/prof.log; [ $rc -eq 0 ] || exit $rc ;;
    prof_td3)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_td3 -o run --output-format csv -- python3 $R/bench.py --algo td3bc --steps 600 --warmup 20 --no-cpu-baseline --transitions 100000 > $R/$OUT/prof_td3.log 2>&1)
      rc=$?; echo "prof rc=$rc" >> $OUT/prof_td3.log; [ $rc -eq 0 ] || exit $rc ;;
    sweep)
      timeout -k 10 300 python tools/gemm_pipeline_sweep.py > $OUT/pipe_sweep.log 2>&1
      rc=$?; [ $rc -eq 0 ] || exit $rc
      timeout -k 10 300 python tools/gemm_pipeline_sweep.py --algo td3 > $OUT/pipe_sweep_td3.log 2>&1
      rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    *) echo "unknown step $STEP"; exit 2 ;;
  esac
done
exit 0

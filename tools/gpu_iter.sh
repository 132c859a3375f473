# iteration run: selected GPU tests ($TESTS), then optional bench lines ($BENCH: ';'-separated arg lists)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-400} python -u -m pytest ${TESTS:-tests} -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/iter_tests.log; [ $rc -eq 0 ] || exit $rc
i=0
IFS=';' read -ra LINES <<< "${BENCH:-}"
for args in "${LINES[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py $args > gpurun_out/iter_bench_$i.log 2>&1 || exit $?
done
exit 0

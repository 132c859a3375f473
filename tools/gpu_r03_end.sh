# Round-end validation of the tree: full GPU suite, smoke(), K2 bench line, K3 bench + breakdown.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/end_tests.log 2>&1; rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/end_smoke.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 2000 --no-cpu-baseline > gpurun_out/end_bench_cql.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --algo bcq --no-cpu-baseline > gpurun_out/end_bench_bcq.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/end_bcq_prof -o run --output-format csv -- python3 bench.py --algo bcq --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/end_bcq_prof.log 2>&1 || exit $?
f=$(find gpurun_out/end_bcq_prof -name '*kernel_trace.csv' -print -quit)
python tools/prof_by_shape.py "$f" 70 > gpurun_out/end_bcq_breakdown.txt 2>&1 || true
rm -f "$f"
exit $rc

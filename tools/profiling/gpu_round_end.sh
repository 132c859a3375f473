# Round-end validation of the committed tree: full GPU suite, smoke(), then the
# round measurement (tools/profiling/gpu_final.sh).  Outputs land in gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/re_gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/re_smoke.log 2>&1 || exit $?
bash tools/profiling/gpu_final.sh

#!/bin/bash
# round 5: the whole GPU suite once + smoke, on the final tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5final
cd $R && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -5 $O/gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
exit $rc

#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5ab
cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_ab_paths.py > $O/ab.log 2>&1; rc=$?
tail -15 $O/ab.log; exit $rc

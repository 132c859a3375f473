#!/bin/bash
# round 5: the arbitrated parity suites with every tensor's margin printed
# (the arbiter's oracles now load private copies of the state: no shared
# optimiser tensors advanced by the fp32 oracle's step before the fp64 ones)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5d
cd $R && mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_cql_parity.py tests/test_gpu_production_path.py tests/test_gpu_dp.py \
  tests/test_gpu_arbiters.py tests/test_gpu_sac_parity.py > $O/arb.log 2>&1
st=$?; tail -3 $O/arb.log; exit $st

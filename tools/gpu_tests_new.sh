# GPU run of the tests added this round (arbiters, K1/K4/K5 parity, API, sampler)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v -s -p no:cacheprovider --timeout 400 --timeout-method thread \
  tests/test_gpu_arbiters.py tests/test_gpu_sampler.py tests/test_golden.py tests/test_online.py \
  > gpurun_out/new_tests.log 2>&1

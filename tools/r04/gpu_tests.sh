# Run a selection of GPU tests: tools/r04/gpu_tests.sh NAME [pytest args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
name=$1; shift
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" \
  > gpurun_out/${name}.log 2>&1

set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/launch_floor.py > gpurun_out/floor.json 2>gpurun_out/floor.err || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/floor_prof -o fl --output-format csv -- python3 tools/launch_floor.py > gpurun_out/floor_prof.log 2>&1 || exit $?

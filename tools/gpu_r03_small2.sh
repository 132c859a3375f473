set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
: > gpurun_out/small_bench.json
for p in 0 1 2 3; do
  D3A_SMALL_PROBE=$p timeout -k 10 120 python3 tools/bench_fwd.py --rows 512 --aux 0 --h-from 0 --bm 16 --n-in 11 --C 1 --J 6 >> gpurun_out/small_bench.json 2>>gpurun_out/small_bench.err || exit $?
done
timeout -k 10 120 python3 tools/bench_fwd.py --rows 512 --aux 0 --h-from 0 --bm 32 --n-in 11 --C 1 --J 6 >> gpurun_out/small_bench.json 2>>gpurun_out/small_bench.err || exit $?

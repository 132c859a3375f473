set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
: > gpurun_out/fwdb.json
for p in 0 1 2 3 4 7; do
  echo "probe $p" >> gpurun_out/fwdb.json
  D3A_FWDB_PROBE=$p timeout -k 10 120 python3 tools/bench_fwd.py --bf16 >> gpurun_out/fwdb.json 2>>gpurun_out/fwdb.err || exit $?
done

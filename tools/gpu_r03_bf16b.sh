set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
: > gpurun_out/bf16b.json
for p in 0 1 2 3 4 7; do
  D3A_BF16_PROBE=$p timeout -k 10 120 python3 tools/bench_bf16.py >> gpurun_out/bf16b.json 2>>gpurun_out/bf16b.err || exit $?
done
bash tools/gpu_r03_bf16.sh

# q2_fwd timing probes on the K2 shape (D3A_FWD_PROBE bits: 1 no h stores,
# 2 register A operand, 4 no epilogue) and the generic kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
: > gpurun_out/fwd3_bench.json
for p in 0 1 2; do
  D3A_FWD_PROBE=$p timeout -k 10 120 python3 tools/bench_fwd.py >> gpurun_out/fwd3_bench.json 2>>gpurun_out/fwd3_bench.err || exit $?
done
D3A_FWD_Q2=0 timeout -k 10 120 python3 tools/bench_fwd.py >> gpurun_out/fwd3_bench.json 2>>gpurun_out/fwd3_bench.err || exit $?

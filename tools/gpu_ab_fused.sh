set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
B="timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-cpu-baseline --transitions 200000"
$B > gpurun_out/ab_bm64.log 2>&1 || exit $?
D3A_FUSED_DIRECT=2 $B > gpurun_out/ab_bm64_wpe1.log 2>&1 || exit $?
D3A_FUSED_DIRECT=3 $B > gpurun_out/ab_bm64_avpipe.log 2>&1 || exit $?
D3A_FUSED_BM=128 $B > gpurun_out/ab_bm128.log 2>&1 || exit $?
for f in gpurun_out/ab_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"avg_launch_us": [0-9.]*' $f)"; done

#!/bin/bash
# round 6: per-launch step timelines of every bench line on the final tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/r6tl
for a in cqldp cqlrepro td3bc bcq dcql; do
  ALGO=$a timeout -k 10 300 bash tools/profiling/gpu_timeline.sh || exit 1
  cp gpurun_out/tl_$a.txt gpurun_out/r6tl/ && cp gpurun_out/tl_$a/run_kernel_stats.csv gpurun_out/r6tl/${a}_kernel_stats.csv
  tail -1 gpurun_out/tl_$a.txt
done

#!/bin/bash
# phase stamps of the K2 x6 critic forward (d3a_q2_fwd_x6, PROBE 16)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5x6st
cd $R && mkdir -p $O
timeout -k 10 200 python -u tools/x6_stamps.py > $O/x6_stamps.txt 2>$O/x6_stamps.err || { tail -20 $O/x6_stamps.err; exit 1; }
cat $O/x6_stamps.txt

#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5sbst
cd $R && mkdir -p $O
D3A_SB_STAMPS=1 timeout -k 10 200 python -u tools/bench_small_bwd.py > $O/st.jsonl 2>$O/st.err || { tail -20 $O/st.err; exit 1; }
timeout -k 10 200 python -u tools/bench_small_bwd.py >> $O/st.jsonl 2>>$O/st.err || { tail -20 $O/st.err; exit 1; }
cat $O/st.jsonl

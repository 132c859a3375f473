#!/bin/bash
# pre-split K2 forward: timing of D3A_X6_PROBE variants (alternating), stamps
# usage: gpu_fwdp.sh TAG "probe1 probe2 ..."
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6fwdp_$1
cd $R && mkdir -p $O
for rep in 1 2 3; do for v in $2; do
  D3A_X6_PROBE=$v timeout -k 10 120 python -u tools/bench_fwd.py --x6 --slice --reps 2000 --warm 1000 --pre >> $O/fwd.jsonl 2>>$O/fwd.err || exit $?
done; done
for v in $3; do
  D3A_X6_PROBE=$v timeout -k 10 120 python -u tools/bench_fwd.py --x6 --slice --stamps --reps 1 --pre >> $O/fwd.jsonl 2>>$O/fwd.err || exit $?
done
python - <<PY
import json
for l in open("$O/fwd.jsonl"):
    d=json.loads(l); print(d["variant"], d["avg_us"], d["max_rel_err_q"], d["stamps"])
PY

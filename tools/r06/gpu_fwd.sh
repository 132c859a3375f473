#!/bin/bash
# K2 forward timing A/B (in-kernel split vs pre-split images) + stamps of the pre-split kernel
# usage: gpu_fwd.sh TAG [extra env for the second arm]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6fwd_$1
cd $R && mkdir -p $O
for v in 0 1 0 1 0 1; do
  P=""; [ $v = 1 ] && P="--pre"
  timeout -k 10 120 python -u tools/bench_fwd.py --x6 --slice --reps 2000 --warm 1000 $P >> $O/fwd.jsonl 2>>$O/fwd.err || exit $?
done
D3A_X6_PROBE=16 timeout -k 10 120 python -u tools/bench_fwd.py --x6 --slice --stamps --reps 1 --pre >> $O/fwd.jsonl 2>>$O/fwd.err || exit $?
python - <<PY
import json
for l in open("$O/fwd.jsonl"):
    d=json.loads(l); print(d["pre"], d["variant"], d["avg_us"], d["max_rel_err_q"], d["stamps"])
PY

#!/bin/bash
# A/B in one call: the BCQ target inside the QR-loss launch against its own launch
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5p
cd $R && mkdir -p $O
: > $O/ab.txt
for v in 1 0 1 0; do
  D3A_BCQ_FUSED_TARGET=$v timeout -k 10 300 python -u bench.py --algo bcq --steps 2000 --warmup 50 --no-cpu-baseline > $O/one.json 2>$O/err.log || { tail -20 $O/err.log; exit 1; }
  python -c "
import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print('fused_target=$v', d['value'], d['ms_per_step'])" | tee -a $O/ab.txt
done

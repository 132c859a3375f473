#!/bin/bash
# the round-5 chunk schedule at XL 32 (K3's narrow-head decoder / residual
# policy passes) against the round-4 one, in one call: BCQ tests, then K3 lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5l
cd $R && mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bcq_parity.py tests/test_gpu_x6.py tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
: > $O/bcq.jsonl
for v in 0 1 0 1; do
  D3A_X6_LEGACY=$v timeout -k 10 300 python -u bench.py --algo bcq --steps 1000 --warmup 50 --no-cpu-baseline >> $O/bcq.jsonl 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bcq.jsonl').read().strip().splitlines()[-1]); print('legacy=$v', d['value'], d['ms_per_step'])"
done

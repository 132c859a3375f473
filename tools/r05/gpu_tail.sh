#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5tail
cd $R && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bcq_parity.py tests/test_gpu_production_path.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 0 1; do
  D3A_BCQ_ADAM_TAIL=$v timeout -k 10 200 python -u bench.py --algo bcq --steps 2000 --warmup 50 --no-cpu-baseline > $O/bench_$v.json 2>$O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('adam_tail=$v', d['value'], d['ms_per_step'])"
done

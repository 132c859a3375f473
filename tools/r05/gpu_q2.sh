#!/bin/bash
# x6 forward change: its tests, then K2 / K3 / K1 bench lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5q2
cd $R && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_x6.py tests/test_gpu_cql_parity.py tests/test_gpu_bcq_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for a in cql; do
  timeout -k 10 200 python -u bench.py --algo $a --steps 1000 --warmup 50 --no-cpu-baseline > $O/bench_$a.json 2>$O/bench_$a.err || { tail -20 $O/bench_$a.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$a.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}
print('$a', d['value'], d['ms_per_step'], r.get('kernel', '')[:40], r.get('avg_launch_us'), r.get('frac'))"
done

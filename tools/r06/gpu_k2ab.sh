#!/bin/bash
# K2 one-call A/B of an env switch: tests (optional), then alternating 2000-step bench lines
# usage: gpu_k2ab.sh TAG VAR "tests..." [algo]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6ab_$1
VAR=$2
ALGO=${4:-cql}
cd $R && mkdir -p $O
if [ -n "$3" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $3 > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for v in 1 0 1 0; do
  env $VAR=$v timeout -k 10 300 python -u bench.py --algo $ALGO --steps 2000 --warmup 50 --no-cpu-baseline > $O/bench_$v.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('$VAR=$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d.get('roofline_other',{}).get('avg_launch_us'))"
done

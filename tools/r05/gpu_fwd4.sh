#!/bin/bash
# K2 forward after the epilogue's bit transpose: timing + stamps, the x6 /
# CQL tests, a K2 bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5r
cd $R && mkdir -p $O
for v in 0 512 1024 0 512 1024; do
  D3A_X6_PROBE=$v timeout -k 10 120 python -u tools/bench_fwd.py --x6 --slice --reps 1000 >> $O/fwd.jsonl 2>>$O/fwd.err || exit $?
done
D3A_X6_PROBE=16 timeout -k 10 120 python -u tools/bench_fwd.py --x6 --slice --stamps --reps 1 >> $O/fwd.jsonl 2>>$O/fwd.err || exit $?
cut -c1-420 $O/fwd.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_x6.py tests/test_gpu_x6t.py tests/test_gpu_cql_parity.py tests/test_gpu_production_path.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 50 --no-cpu-baseline > $O/bench_cql.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_cql.json').read().strip().splitlines()[-1]); print('cql', d['value'], d['ms_per_step'], d.get('roofline',{}).get('achieved'))"

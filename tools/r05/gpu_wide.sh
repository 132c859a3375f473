#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5wide
cd $R && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_x6.py tests/test_gpu_bcq_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ABLS=0 D3A_WIDE_STAMPS=1 timeout -k 10 200 python -u tools/bench_wide.py > $O/wide.json 2>$O/wide.err || { tail -20 $O/wide.err; exit 1; }
python -c "
import json; d=json.load(open('$O/wide.json'))
for k,v in d.items():
    if k.startswith('abl'): print(k, v['avg_us'], v['phase_cycles_mean'], v['tile_cycles_mean'], v['wg_cycles_mean'], v['wg_cycles_max'])
"
timeout -k 10 200 python -u bench.py --algo bcq --steps 300 --warmup 50 --no-cpu-baseline > $O/bench_bcq.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_bcq.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"

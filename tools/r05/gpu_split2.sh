#!/bin/bash
# the paired split (x6.hpp split2): K2 forward timing + stamps, the wide
# kernel's stamps, the whole GPU suite, then K2 / K3 bench lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r5h
cd $R && mkdir -p $O
for v in 0 64; do
  D3A_X6_PROBE=$v timeout -k 10 120 python -u tools/bench_fwd.py --x6 --slice --reps 1000 >> $O/fwd.jsonl 2>>$O/fwd.err || exit $?
done
D3A_X6_PROBE=16 timeout -k 10 120 python -u tools/bench_fwd.py --x6 --slice --stamps --reps 1 >> $O/fwd.jsonl 2>>$O/fwd.err || exit $?
cut -c1-420 $O/fwd.jsonl
ABLS=0 D3A_WIDE_STAMPS=1 timeout -k 10 200 python -u tools/bench_wide.py > $O/wide.json 2>$O/wide.err || { tail -20 $O/wide.err; exit 1; }
python -c "
import json; d=json.load(open('$O/wide.json'))
for k,v in d.items():
    if k.startswith('abl'): print(k, v['avg_us'], v['phase_cycles_mean'], v['tile_cycles_mean'])
"
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 50 --no-cpu-baseline > $O/bench_cql.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_cql20.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --algo bcq --steps 300 --warmup 50 --no-cpu-baseline > $O/bench_bcq.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
for f in cql cql20 bcq; do python -c "
import json; d=json.loads(open('$O/bench_$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('roofline',{}).get('achieved'))"; done

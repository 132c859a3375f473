#!/bin/bash
# pre-split forward: stamps + SQ counters (VALU / MFMA), op-replay test, K2 A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r6b
cd $R && mkdir -p $O
export TMPDIR=/tmp
for P in "" "--pre"; do
  D3A_X6_PROBE=16 timeout -k 10 120 python -u tools/bench_fwd.py --x6 --slice --stamps --reps 1 $P >> $O/stamps.jsonl 2>>$O/fwd.err || exit $?
done
cut -c1-600 $O/stamps.jsonl
cd /tmp
for P in "" "--pre"; do
  n=sq${P#--}
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d $O/$n -o run --output-format csv -- python3 $R/tools/bench_fwd.py --x6 --slice --reps 50 $P > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  (cd $R && python tools/pmc_sq_summary.py $O/$n q2x6_fwd > $O/r06_pmc_sq_k2_fwd$P.txt; cat $O/r06_pmc_sq_k2_fwd$P.txt)
  find $O -name "*counter_collection.csv" -size +20M -delete
done
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_torch_ops.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0 1 0; do
  D3A_X6_PRESPLIT=$v timeout -k 10 300 python -u bench.py --steps 2000 --warmup 50 --no-cpu-baseline > $O/bench_$v.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('presplit=$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
for v in 1 0 1 0; do
  D3A_OP_REPLAY=$v timeout -k 10 300 python -u bench.py --steps 2000 --warmup 50 --no-cpu-baseline > $O/bench_op$v.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_op$v.json').read().strip().splitlines()[-1]); print('op_replay=$v', d['value'], d['ms_per_step'], d['host']['host_us_per_step'])"
done
